"""Evaluation CLI — drop-in for the reference eval.py (same flags, filenames and figure layout).

Builds the DPT ``Transformer`` (models/net.py), loads the checkpoint with the
safe tensor-only loader, and dispatches to evals/* whose hot loops run on the
MI355X kernels of libdpt_hip.so.
"""
import argparse
import os
import pickle
import time

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402

import common_args  # noqa: E402
from evals import eval_bandit, eval_darkroom, eval_linear_bandit  # noqa: E402
from models.net import Transformer  # noqa: E402
from utils import (build_bandit_data_filename, build_bandit_model_filename,  # noqa: E402
                   build_darkroom_data_filename, build_darkroom_model_filename,
                   build_linear_bandit_data_filename, build_linear_bandit_model_filename)

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def load_checkpoint(model, path):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(sd)
    return model


def main(argv=None):
    parser = argparse.ArgumentParser()
    common_args.add_dataset_args(parser)
    common_args.add_model_args(parser)
    common_args.add_eval_args(parser)
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--checkpoint", type=str, default=None,
                        help="Path to checkpoint file; if set, overrides default model path")
    args = vars(parser.parse_args(argv))
    print("Args: ", args)

    H, dim = args["H"], args["dim"]
    state_dim, action_dim = dim, dim
    envname, seed, epoch = args["env"], args["seed"], args["epoch"]
    var, cov, lin_d = args["var"], args["cov"], args["lin_d"]
    horizon = args["hor"] if args["hor"] >= 0 else H
    test_cov = args["test_cov"] if args["test_cov"] >= 0 else cov
    n_eval = args["n_eval"]
    tmp_seed = 0 if seed == -1 else seed
    torch.manual_seed(tmp_seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(tmp_seed)
    np.random.seed(tmp_seed)

    model_config = {"shuffle": args["shuffle"], "lr": args["lr"], "dropout": args["dropout"], "n_embd": args["embd"],
                    "n_layer": args["layer"], "n_head": args["head"], "n_envs": args["envs"], "n_hists": args["hists"],
                    "n_samples": args["samples"], "horizon": horizon, "dim": dim, "seed": seed}
    bandit_type = "uniform"
    if envname in ("bandit", "bandit_bernoulli"):
        state_dim = 1
        model_config.update({"var": var, "cov": cov})
        filename = build_bandit_model_filename(envname, model_config)
        bandit_type = "uniform" if envname == "bandit" else "bernoulli"
    elif envname == "linear_bandit":
        state_dim = 1
        model_config.update({"lin_d": lin_d, "var": var, "cov": cov})
        filename = build_linear_bandit_model_filename(envname, model_config)
    elif envname.startswith("darkroom"):
        state_dim, action_dim = 2, 5
        filename = build_darkroom_model_filename(envname, model_config)
    else:
        raise NotImplementedError(f"{envname} (miniworld is out of scope)")

    config = {"horizon": H, "state_dim": state_dim, "action_dim": action_dim, "n_layer": args["layer"],
              "n_embd": args["embd"], "n_head": args["head"], "dropout": args["dropout"], "test": True}
    model = Transformer(config).to(device)
    if args["checkpoint"] is not None:
        model_path = args["checkpoint"]
    elif epoch < 0:
        model_path = f"trained_models/{filename}.pt"
    else:
        model_path = f"trained_models/{filename}_epoch{epoch}.pt"
    load_checkpoint(model, model_path)
    model.eval()

    dataset_config = {"horizon": horizon, "dim": dim}
    if envname in ("bandit", "bandit_bernoulli"):
        dataset_config.update({"var": var, "cov": cov, "type": "uniform"})
        eval_filepath = build_bandit_data_filename(envname, n_eval, dataset_config, mode=2)
        save_filename = f"{filename}_testcov{test_cov}_hor{horizon}.pkl"
    elif envname == "linear_bandit":
        dataset_config.update({"lin_d": lin_d, "var": var, "cov": cov})
        eval_filepath = build_linear_bandit_data_filename(envname, n_eval, dataset_config, mode=2)
        save_filename = f"{filename}_testcov{test_cov}_hor{horizon}.pkl"
    else:
        dataset_config.update({"rollin_type": "uniform"})
        eval_filepath = build_darkroom_data_filename(envname, n_eval, dataset_config, mode=2)
        save_filename = f"{filename}_hor{horizon}.pkl"
    # datasets are our own pickles (collect_data.py output), as in the reference
    with open(eval_filepath, "rb") as f:
        eval_trajs = pickle.load(f)
    n_eval = min(n_eval, len(eval_trajs))

    evals_filename = f"evals_epoch{epoch}"
    for sub in ("", "/bar", "/online", "/graph"):
        os.makedirs(f"figs/{evals_filename}{sub}", exist_ok=True)
    t0 = time.time()
    if envname in ("bandit", "bandit_bernoulli"):
        cfg = {"horizon": horizon, "var": var, "n_eval": n_eval, "bandit_type": bandit_type}
        eval_bandit.online(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/online/{save_filename}.png")
        plt.clf(), plt.cla(), plt.close()
        eval_bandit.offline(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/bar/{save_filename}_bar.png")
        plt.clf()
        eval_bandit.offline_graph(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/graph/{save_filename}_graph.png")
        plt.clf()
    elif envname == "linear_bandit":
        cfg = {"horizon": horizon, "var": var, "n_eval": n_eval}
        eval_linear_bandit.online(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/online/{save_filename}.png")
        plt.clf(), plt.cla(), plt.close()
        eval_linear_bandit.offline(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/bar/{save_filename}_bar.png")
        plt.clf()
        eval_linear_bandit.offline_graph(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/graph/{save_filename}_graph.png")
        plt.clf()
    else:
        cfg = {"Heps": 40, "horizon": horizon, "H": H, "n_eval": min(20, n_eval), "dim": dim,
               "permuted": envname == "darkroom_permuted"}
        eval_darkroom.online(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/online/{save_filename}.png")
        plt.clf()
        del cfg["Heps"], cfg["horizon"]
        cfg["n_eval"] = n_eval
        eval_darkroom.offline(eval_trajs, model, **cfg)
        plt.savefig(f"figs/{evals_filename}/bar/{save_filename}_bar.png")
        plt.clf()
    print(f"Evaluation took {time.time() - t0:.2f} s")


if __name__ == "__main__":
    main()
