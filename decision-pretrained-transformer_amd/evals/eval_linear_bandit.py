"""Linear-bandit evaluation — drop-in for the reference evals/eval_linear_bandit.py.

The online loop is the same as the Gaussian bandit's (eval_linear_bandit.py:54-97
is a verbatim copy of eval_bandit.py:56-103), so it reuses the fused device
rollout; only the task construction (LinearBanditEnv: means = arms @ theta)
differs.
"""
import numpy as np
import torch

from ctrls.ctrl_bandit import BanditTransformerController, OptPolicy
from envs.bandit_env import BanditEnvVec, LinearBanditEnv
from evals.eval_bandit import deploy_online, deploy_online_vec, regret_stats  # noqa: F401

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _envs(eval_trajs, n_eval, horizon, var):
    return [LinearBanditEnv(eval_trajs[i]["theta"], eval_trajs[i]["arms"], horizon, var=var) for i in range(n_eval)]


def online(eval_trajs, model, n_eval, horizon, var):
    """evals/eval_linear_bandit.py:101-199 (Opt + DPT learner; TS / LinUCB when built)."""
    import matplotlib.pyplot as plt
    envs = _envs(eval_trajs, n_eval, horizon, var)
    vec_env = BanditEnvVec(envs)
    all_means = {"opt": deploy_online_vec(vec_env, OptPolicy(envs, batch_size=len(envs)), horizon).T}
    ctrl = BanditTransformerController(model, sample=True, batch_size=len(envs))
    all_means["Lnr"] = deploy_online_vec(vec_env, ctrl, horizon).T
    from ctrls import ctrl_bandit as cb
    if hasattr(cb, "LinUCBPolicy"):
        all_means["LinUCB"] = deploy_online_vec(vec_env, cb.LinUCBPolicy(envs[0], const=1.0, batch_size=len(envs)),
                                                horizon).T
    if hasattr(cb, "ThompsonSamplingPolicy"):
        ts = cb.ThompsonSamplingPolicy(envs[0], std=var, sample=True, prior_mean=0.0, prior_var=1.0,
                                       warm_start=False, batch_size=len(envs))
        all_means["Thomp"] = deploy_online_vec(vec_env, ts, horizon).T
    st = regret_stats(all_means)
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(15, 6))
    for key, m in st["means"].items():
        ax1.plot(m, label=key)
    ax1.set_yscale("log")
    ax1.legend()
    for key, m in st["regret_means"].items():
        if key != "opt":
            ax2.plot(m, label=key)
    ax2.legend()
    return all_means, st


def offline(eval_trajs, model, n_eval, horizon, var):
    """evals/eval_linear_bandit.py:202-286 (Opt + DPT greedy on a fixed context)."""
    import matplotlib.pyplot as plt
    envs = _envs(eval_trajs, n_eval, horizon, var)
    vec_env = BanditEnvVec(envs)
    batch = {"context_states": np.stack([t["context_states"][:horizon] for t in eval_trajs[:n_eval]]),
             "context_actions": np.stack([t["context_actions"][:horizon] for t in eval_trajs[:n_eval]]),
             "context_next_states": np.stack([t["context_next_states"][:horizon] for t in eval_trajs[:n_eval]]),
             "context_rewards": np.stack([t["context_rewards"][:horizon, None] for t in eval_trajs[:n_eval]])}
    opt = OptPolicy(envs, batch_size=n_eval)
    lnr = BanditTransformerController(model, sample=False, batch_size=n_eval)
    opt.set_batch_numpy_vec(batch)
    lnr.set_batch_numpy_vec(batch)
    baselines = {"opt": np.array(vec_env.deploy_eval(opt)[3]), "lnr": np.array(vec_env.deploy_eval(lnr)[3])}
    means = {k: np.mean(v) for k, v in baselines.items()}
    plt.bar(means.keys(), means.values())
    return baselines


def offline_graph(eval_trajs, model, n_eval, horizon, var):
    import matplotlib.pyplot as plt
    horizons = np.linspace(1, horizon, 50, dtype=int)
    all_means = []
    for h in horizons:
        b = offline(eval_trajs, model, n_eval=n_eval, horizon=h, var=var)
        plt.clf()
        all_means.append({k: np.mean(v) for k, v in b.items()})
    for key in all_means[0]:
        if key != "opt":
            plt.plot(horizons, [m["opt"] - m[key] for m in all_means], label=key)
    plt.legend()
    plt.yscale("log")
    return horizons, all_means
