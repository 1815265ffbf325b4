"""Filename builders and tensor conversion — drop-in for the reference utils.py.

The reference encodes each dataset / model configuration into its filename
(utils.py:14-190); the same names are produced here so datasets and
checkpoints are interchangeable with the reference's.  The builders are
table-driven: one ordered list of (suffix, config key) per family.
"""
import numpy as np
import torch

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")

_MODE_SUFFIX = {0: "_train", 1: "_test"}

# ordered (suffix, key) fields after the env name, per family
_DATA_FIELDS = {
    "bandit": [("_H", "horizon"), ("_d", "dim"), ("_var", "var"), ("_cov", "cov")],
    "linear_bandit": [("_H", "horizon"), ("_d", "dim"), ("_lind", "lin_d"), ("_var", "var"), ("_cov", "cov")],
    "darkroom": [("_H", "horizon"), ("_d", "dim")],
}
_MODEL_HEAD = [("_shuf", "shuffle"), ("_lr", "lr"), ("_do", "dropout"), ("_embd", "n_embd"), ("_layer", "n_layer"),
               ("_head", "n_head"), ("_envs", "n_envs"), ("_hists", "n_hists"), ("_samples", "n_samples")]
_MODEL_TAIL = {
    "bandit": [("_var", "var"), ("_cov", "cov"), ("_H", "horizon"), ("_d", "dim"), ("_seed", "seed")],
    "linear_bandit": [("_var", "var"), ("_cov", "cov"), ("_H", "horizon"), ("_d", "dim"), ("_lind", "lin_d"),
                      ("_seed", "seed")],
    "darkroom": [("_H", "horizon"), ("_d", "dim"), ("_seed", "seed")],
}


def _fields(config, fields):
    return "".join(suffix + str(config[key]) for suffix, key in fields)


def _data_filename(family, env, n_envs, config, mode):
    name = f"{env}_envs{n_envs}"
    if mode != 2:
        name += f"_hists{config['n_hists']}_samples{config['n_samples']}"
    name += _fields(config, _DATA_FIELDS[family])
    if mode == 2:
        if family == "darkroom":
            name += "_" + config["rollin_type"]
        name += "_eval"
    else:
        name += _MODE_SUFFIX.get(mode, "")
    return f"datasets/trajs_{name}.pkl"


def _model_filename(family, env, config):
    return env + _fields(config, _MODEL_HEAD) + _fields(config, _MODEL_TAIL[family])


def build_bandit_data_filename(env, n_envs, config, mode):
    """Mode 0: train, 1: test, 2: eval (utils.py:14-37)."""
    return _data_filename("bandit", env, n_envs, config, mode)


def build_bandit_model_filename(env, config):
    return _model_filename("bandit", env, config)


def build_linear_bandit_data_filename(env, n_envs, config, mode):
    return _data_filename("linear_bandit", env, n_envs, config, mode)


def build_linear_bandit_model_filename(env, config):
    return _model_filename("linear_bandit", env, config)


def build_darkroom_data_filename(env, n_envs, config, mode):
    return _data_filename("darkroom", env, n_envs, config, mode)


def build_darkroom_model_filename(env, config):
    return _model_filename("darkroom", env, config)


def convert_to_tensor(x, store_gpu=True):
    """numpy/list -> float32 tensor, on the device by default (utils.py:193-197)."""
    t = torch.tensor(np.asarray(x)).float()
    return t.to(device) if store_gpu else t


def worker_init_fn(worker_id):
    worker_seed = torch.initial_seed() % (2 ** 32) + worker_id
    torch.manual_seed(worker_seed)
    np.random.seed(int(worker_seed % (2 ** 32 - 1)))
