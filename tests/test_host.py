"""Host-side drop-in surface on CPU: filenames and CLI flags equal the reference's
(tests/golden/host_surface.json, recorded from the reference's utils.py / common_args.py)."""
import argparse
import json
import os

from conftest import GOLDEN


def surface():
    return json.load(open(os.path.join(GOLDEN, "host_surface.json")))


def test_filenames_match_reference():
    import utils
    for fn, args, expected in surface()["filenames"]:
        assert getattr(utils, fn)(*args) == expected, (fn, args)


def test_flag_defaults_match_reference():
    import common_args
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_train_args(p)
    common_args.add_eval_args(p)
    assert vars(p.parse_args(["--env", "bandit"])) == surface()["defaults"]


def test_run_scripts_parse():
    """The reference recipes' collect / eval command lines parse with our CLIs (run_bandit.sh:2,8)."""
    import common_args
    collect = "--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --envs_eval 200".split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    a = vars(p.parse_args(collect))
    assert a["H"] == 500 and a["envs_eval"] == 200
    ev = ("--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --lr 0.0001 --layer 4 --head 4 "
          "--shuffle --epoch 50 --n_eval 200 --seed 1").split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_eval_args(p)
    p.add_argument("--seed", type=int, default=0)
    a = vars(p.parse_args(ev))
    assert a["shuffle"] is True and a["layer"] == 4 and a["epoch"] == 50


def _tiny_transformer():
    from models.net import Transformer
    return Transformer(dict(horizon=4, state_dim=1, action_dim=5, n_layer=2, n_embd=32, n_head=1, dropout=0.0,
                            test=False))


def _tiny_batch():
    import torch
    return {"query_states": torch.ones(2, 1), "zeros": torch.zeros(2, 7), "context_states": torch.ones(2, 3, 1),
            "context_actions": torch.eye(5)[[0, 1, 2]].expand(2, 3, 5), "context_next_states": torch.ones(2, 3, 1),
            "context_rewards": torch.zeros(2, 3, 1)}


def test_training_forward_takes_the_hip_training_path():
    """train.py:286-331 (model in training mode, grad enabled) routes the forward through the HIP
    training kernels (dpt_hip.train.TransformerFunction, whose backward fills every parameter's
    .grad); on this CPU-only container that path refuses to run because there is no GPU."""
    import pytest
    m = _tiny_transformer()
    assert m.training
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        m(_tiny_batch())


def test_train_blob_order_matches_pack_weights():
    """dpt_hip.train.pack_params (the device-side pack of the training path) lays the parameters
    out exactly as dpt_hip.pack_weights (the inference blob of include/dpt_hip.h), and
    unpack_grads inverts it shape for shape."""
    import torch
    import dpt_hip
    from dpt_hip import train as tr
    m = _tiny_transformer()
    ps = tr.param_list(m)
    sd = {k: v for k, v in m.state_dict().items() if not k.endswith("wte.weight")}
    assert torch.equal(tr.pack_params(ps), dpt_hip.pack_weights(sd, m.n_layer))
    assert len(ps) == len(sd) and sum(p.numel() for p in ps) == sum(v.numel() for v in sd.values())
    back = tr.unpack_grads(tr.pack_params(ps), ps)
    assert all(torch.equal(a, b) for a, b in zip(back, ps))


def test_training_mode_dropout_is_rejected():
    """GPT2Config applies dropout in training mode (models/net.py:30-32); the HIP kernels have none,
    so a training-mode forward with dropout > 0 raises (with or without grad) instead of training
    or evaluating without it.  Eval mode ignores dropout, as the reference does."""
    import pytest
    import torch
    from models.net import Transformer
    m = Transformer(dict(horizon=4, state_dim=1, action_dim=5, n_layer=2, n_embd=32, n_head=1, dropout=0.1,
                         test=False))
    with pytest.raises(NotImplementedError, match="dropout"):
        m(_tiny_batch())
    with torch.no_grad(), pytest.raises(NotImplementedError, match="dropout"):
        m(_tiny_batch())
    m.eval()
    with pytest.raises(RuntimeError, match="ROCm GPU"):  # eval mode goes on to the (absent) GPU
        m(_tiny_batch())
