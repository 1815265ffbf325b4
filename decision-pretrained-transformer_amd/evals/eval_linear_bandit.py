"""Linear-bandit evaluation — drop-in for the reference evals/eval_linear_bandit.py.

The online loop is the same as the Gaussian bandit's (eval_linear_bandit.py:54-97
is a verbatim copy of eval_bandit.py:56-103), so it reuses the fused device
rollout; only the task construction (LinearBanditEnv: means = arms @ theta) and
the comparison policies differ: Thompson sampling with a N(0, 1) prior and
LinUCB (ctrls/ctrl_bandit.py:447-528, dpt_rollout_policy) online; the 100-draw
Thompson vote and LinUCB with const 0 ("linreg") offline.
"""
import numpy as np
import torch

from ctrls.ctrl_bandit import BanditTransformerController, LinUCBPolicy, OptPolicy, ThompsonSamplingPolicy
from envs.bandit_env import BanditEnvVec, LinearBanditEnv
from evals.eval_bandit import deploy_online, deploy_online_vec, regret_stats  # noqa: F401

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def _envs(eval_trajs, n_eval, horizon, var):
    return [LinearBanditEnv(eval_trajs[i]["theta"], eval_trajs[i]["arms"], horizon, var=var) for i in range(n_eval)]


def online(eval_trajs, model, n_eval, horizon, var):
    """evals/eval_linear_bandit.py:101-199: Opt, the DPT learner, Thompson (prior 0 / 1), LinUCB
    (const 1), in the reference's order (each controller draws its Philox seed from numpy's global
    RNG at its first step, as the reference's controllers draw from it, so the order fixes the
    draws), then the suboptimality and cumulative-regret
    curves."""
    import matplotlib.pyplot as plt
    envs = _envs(eval_trajs, n_eval, horizon, var)
    vec_env = BanditEnvVec(envs)
    n = len(envs)
    all_means = {"opt": deploy_online_vec(vec_env, OptPolicy(envs, batch_size=n), horizon).T}
    all_means["Lnr"] = deploy_online_vec(vec_env, BanditTransformerController(model, sample=True, batch_size=n),
                                         horizon).T
    ts = ThompsonSamplingPolicy(envs[0], std=var, sample=True, prior_mean=0.0, prior_var=1.0, warm_start=False,
                                batch_size=n)
    all_means["Thomp"] = deploy_online_vec(vec_env, ts, horizon).T
    all_means["LinUCB"] = deploy_online_vec(vec_env, LinUCBPolicy(envs[0], const=1.0, batch_size=n), horizon).T
    for v in all_means.values():
        assert v.shape[0] == n_eval
    st = regret_stats(all_means)
    fig, (ax1, ax2) = plt.subplots(1, 2, figsize=(15, 6))
    for key, m in st["means"].items():
        s = st["sems"][key]
        if key == "opt":
            ax1.plot(m, label=key, linestyle="--", color="black", linewidth=2)
            ax1.fill_between(np.arange(horizon), m - s, m + s, alpha=0.2, color="black")
        else:
            ax1.plot(m, label=key)
            ax1.fill_between(np.arange(horizon), m - s, m + s, alpha=0.2)
    ax1.set_yscale("log")
    ax1.set_xlabel("Episodes")
    ax1.set_ylabel("Suboptimality")
    ax1.set_title("Online Evaluation")
    ax1.legend()
    for key, m in st["regret_means"].items():
        if key != "opt":
            s = st["regret_sems"][key]
            ax2.plot(m, label=key)
            ax2.fill_between(np.arange(horizon), m - s, m + s, alpha=0.2)
    ax2.set_xlabel("Episodes")
    ax2.set_ylabel("Cumulative Regret")
    ax2.set_title("Regret Over Time")
    ax2.legend()
    return all_means, st


def offline(eval_trajs, model, n_eval, horizon, var):
    """evals/eval_linear_bandit.py:202-286: on the first ``horizon`` transitions of each task's
    context (rewards deterministic, BanditEnvVec.deploy_eval), the rewards of Opt, the DPT greedy
    leg, the Thompson 100-draw vote (prior 0 / 1) and LinUCB with const 0 ("linreg", the
    ridge-regression arm), keyed as the reference keys them."""
    import matplotlib.pyplot as plt
    envs = _envs(eval_trajs, n_eval, horizon, var)
    vec_env = BanditEnvVec(envs)
    sl = eval_trajs[:n_eval]
    batch = {"context_states": np.stack([t["context_states"][:horizon] for t in sl]),
             "context_actions": np.stack([t["context_actions"][:horizon] for t in sl]),
             "context_next_states": np.stack([t["context_next_states"][:horizon] for t in sl]),
             "context_rewards": np.stack([np.asarray(t["context_rewards"])[:horizon, None] for t in sl])}
    opt_policy = OptPolicy(envs, batch_size=n_eval)
    lnr_policy = BanditTransformerController(model, sample=False, batch_size=n_eval)
    thomp_policy = ThompsonSamplingPolicy(envs[0], std=var, sample=False, prior_mean=0, prior_var=1.0,
                                          warm_start=False, batch_size=n_eval)
    linreg_policy = LinUCBPolicy(envs[0], const=0.0, batch_size=n_eval)
    for pol in (opt_policy, thomp_policy, lnr_policy, linreg_policy):
        pol.set_batch_numpy_vec(batch)
    baselines = {"opt": np.array(vec_env.deploy_eval(opt_policy)[3]),
                 "lnr": np.array(vec_env.deploy_eval(lnr_policy)[3]),
                 "thmp": np.array(vec_env.deploy_eval(thomp_policy)[3]),
                 "linreg": np.array(vec_env.deploy_eval(linreg_policy)[3])}
    means = {k: np.mean(v) for k, v in baselines.items()}
    colors = plt.cm.viridis(np.linspace(0, 1, len(means)))
    plt.bar(means.keys(), means.values(), color=colors)
    plt.title(f"Mean Reward on {n_eval} Trajectories")
    return baselines


def offline_graph(eval_trajs, model, n_eval, horizon, var):
    """evals/eval_linear_bandit.py:289-339: offline() at every context length 1..horizon
    (np.linspace(1, horizon, horizon)), suboptimality mean / SEM per leg against dataset size.
    Returns the context lengths and offline()'s result at each."""
    import matplotlib.pyplot as plt
    import scipy.stats
    horizons = np.linspace(1, horizon, horizon, dtype=int)
    all_baselines, all_subopt_means, all_subopt_sems = [], [], []
    for h in horizons:
        baselines = offline(eval_trajs, model, n_eval=n_eval, horizon=h, var=var)
        plt.clf()
        subopt = {k: baselines["opt"] - v for k, v in baselines.items()}
        all_baselines.append(baselines)
        all_subopt_means.append({k: np.mean(v) for k, v in subopt.items()})
        all_subopt_sems.append({k: scipy.stats.sem(v) for k, v in subopt.items()})
    for key in all_baselines[-1]:
        if key != "opt":
            m = np.array([s[key] for s in all_subopt_means])
            e = np.array([s[key] for s in all_subopt_sems])
            plt.plot(horizons, m, label=key)
            plt.fill_between(horizons, m - e, m + e, alpha=0.2)
    plt.legend()
    plt.yscale("log")
    plt.xlabel("Dataset size")
    plt.ylabel("Suboptimality")
    return horizons, all_baselines
