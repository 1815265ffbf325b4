"""Bandit evaluation — drop-in for the reference evals/eval_bandit.py.

``deploy_online_vec`` (evals/eval_bandit.py:56-103) is THE hot loop: when the
controller is the DPT ``BanditTransformerController`` over this package's
``Transformer`` and the env is ``BanditEnvVec``, the entire H-step loop runs as
ONE gfx950 kernel launch (dpt_rollout_bandit: exact K/V-cache decode + device
sampling + env step + context append), returning the same ``cum_means``
(H, N) fp64 array and ``meta`` contexts as the reference.  Any other
controller runs the reference's per-step loop unchanged (envs still step on
the device).
"""
import numpy as np
import torch

import dpt_hip
from ctrls.ctrl_bandit import BanditTransformerController, OptPolicy
from envs.bandit_env import BanditEnv, BanditEnvVec
from utils import convert_to_tensor

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def deploy_online(env, controller, horizon):
    """Single-env online loop (evals/eval_bandit.py:24-53)."""
    dev = dpt_hip.device()
    context_states = torch.zeros((1, horizon, env.dx), device=dev)
    context_actions = torch.zeros((1, horizon, env.du), device=dev)
    context_next_states = torch.zeros((1, horizon, env.dx), device=dev)
    context_rewards = torch.zeros((1, horizon, 1), device=dev)
    cum_means = []
    for h in range(horizon):
        batch = {"context_states": context_states[:, :h, :], "context_actions": context_actions[:, :h, :],
                 "context_next_states": context_next_states[:, :h, :], "context_rewards": context_rewards[:, :h, :]}
        controller.set_batch(batch)
        states_lnr, actions_lnr, next_states_lnr, rewards_lnr = env.deploy(controller)
        context_states[0, h, :] = convert_to_tensor(states_lnr[0])
        context_actions[0, h, :] = convert_to_tensor(actions_lnr[0])
        context_next_states[0, h, :] = convert_to_tensor(next_states_lnr[0])
        context_rewards[0, h, :] = convert_to_tensor(rewards_lnr[0])
        cum_means.append(env.get_arm_value(actions_lnr.flatten()))
    return np.array(cum_means)


def _fused_ok(vec_env, controller, horizon):
    """The one-launch rollout: our controller, env and model, with no dropout in play (a
    training-mode model with dropout > 0 takes the per-step loop, whose forward applies it)."""
    from models.net import Transformer
    if not (isinstance(controller, BanditTransformerController) and isinstance(vec_env, BanditEnvVec)):
        return False
    m = controller.model
    return (isinstance(m, Transformer) and m.state_dim == 1 and not (m.training and m.dropout > 0)
            and controller.batch_size == vec_env.num_envs and horizon <= m.n_positions)


def rollout_fused(vec_env, controller, horizon, uniforms=None, noise=None, seed=None, first_task=None):
    """One-launch online rollout; returns the device result dict of DeviceModel.rollout_bandit.

    Selection draws are the controller's own stream, as in the per-step path
    (BanditTransformerController._select): the H counters that loop would consume
    one per step are consumed here in one go, so both paths act on the same
    Philox draws, and uniforms injected on the controller (``controller.uniforms``)
    are used unless ``uniforms`` is given explicitly.  Draws are keyed by the
    global task id (``vec_env.first_task`` for a shard).
    """
    s0, ctr0 = controller._stream.next()
    controller._stream.counter = ctr0 + horizon
    seed = s0 if seed is None else seed
    if uniforms is None and controller.sample and controller.uniforms is not None:
        uniforms = np.stack([np.asarray(controller.uniforms(ctr0 + h), dtype=np.float64).reshape(-1)
                             for h in range(horizon)])
    if first_task is None:
        first_task = getattr(vec_env, "first_task", 0)
    kw = dict(seed=seed, first_task=first_task, uniforms=uniforms, noise=noise, counter=ctr0)
    model = controller.model
    if model.n_embd != dpt_hip.E:  # widths the fused kernel is not built for: the generic-width rollout
        from dpt_hip import train as tr
        return tr.rollout_bandit_generic(model, vec_env.means_device, horizon, vec_env.var, controller.sample,
                                         vec_env.type_code, **kw)
    return model.device_model().rollout_bandit(vec_env.means_device, horizon, vec_env.var, controller.sample,
                                               vec_env.type_code, **kw)


def _policy_ok(vec_env, controller):
    from ctrls.ctrl_bandit import _KernelPolicy
    return (isinstance(vec_env, BanditEnvVec) and isinstance(controller, (_KernelPolicy, OptPolicy))
            and getattr(controller, "batch_size", vec_env.num_envs) == vec_env.num_envs)


def rollout_policy_fused(vec_env, controller, horizon, noise=None, policy_noise=None, seed=None, first_task=None):
    """One-launch rollout of a classical controller (dpt_rollout_policy).  The policy's draws
    come from the controller's stream as in its per-step act_numpy_vec (the H counters that
    loop would consume are consumed here in one go), or from ``controller.policy_noise``;
    keyed by the global task id (``vec_env.first_task`` for a shard)."""
    ctr0 = 0
    if isinstance(controller, OptPolicy):
        code, kw = dpt_hip.POLICY_OPT, {}
        s0 = dpt_hip.next_seed()
    else:
        code, kw = controller.policy, controller.kernel_kwargs()
        s0, ctr0 = controller._stream.next()
        controller._stream.counter = ctr0 + horizon
        if policy_noise is None and controller.policy_noise is not None:
            policy_noise = np.stack([np.asarray(controller.policy_noise(ctr0 + h), np.float64)
                                     for h in range(horizon)])
    seed = s0 if seed is None else seed
    if first_task is None:
        first_task = getattr(vec_env, "first_task", 0)
    return dpt_hip.rollout_policy(code, vec_env.means_device, horizon, vec_env.var, vec_env.type_code, seed=seed,
                                  first_task=first_task, noise=noise, policy_noise=policy_noise, counter=ctr0, **kw)


def deploy_online_vec(vec_env, controller, horizon, include_meta=False, uniforms=None, noise=None,
                      policy_noise=None, fused=True):
    """evals/eval_bandit.py:56-103.  ``uniforms``/``noise`` (H, N) optionally inject the
    selection uniforms / reward normals (reproduces a reference run draw for draw);
    ``policy_noise`` the classical policies' own draws (Thompson posterior normals).
    ``fused=False`` forces the reference's per-step loop."""
    num_envs = vec_env.num_envs
    out = None
    if fused and _fused_ok(vec_env, controller, horizon):
        out = rollout_fused(vec_env, controller, horizon, uniforms, noise)
    elif fused and _policy_ok(vec_env, controller):
        out = rollout_policy_fused(vec_env, controller, horizon, noise, policy_noise)
    if out is not None:
        cum_means = out["arm_value"].t().cpu().numpy()
        if not include_meta:
            return cum_means
        acts = out["actions"].cpu().numpy()
        meta = {"context_states": np.ones((num_envs, horizon, vec_env.dx)),
                "context_actions": np.eye(vec_env.du)[acts],
                "context_next_states": np.ones((num_envs, horizon, vec_env.dx)),
                "context_rewards": out["rewards"].cpu().numpy()[..., None]}
        return cum_means, meta

    # the reference's per-step loop; injected draws are handed to the env / controller hooks
    # (step h uses row h), which read them by their own stream counters
    hooks = []

    def hook(obj, attr, rows):
        if rows is not None and hasattr(obj, attr):
            c0 = obj._stream.counter
            hooks.append((obj, attr, getattr(obj, attr)))
            setattr(obj, attr, lambda k, _r=rows, _c=c0: _r[k - _c])

    hook(vec_env, "noise", noise)
    hook(controller, "uniforms", uniforms)
    hook(controller, "policy_noise", policy_noise)
    try:
        return _deploy_online_steps(vec_env, controller, horizon, include_meta)
    finally:
        for obj, attr, old in hooks:
            setattr(obj, attr, old)


def _deploy_online_steps(vec_env, controller, horizon, include_meta):
    num_envs = vec_env.num_envs
    context_states = np.zeros((num_envs, horizon, vec_env.dx))
    context_actions = np.zeros((num_envs, horizon, vec_env.du))
    context_next_states = np.zeros((num_envs, horizon, vec_env.dx))
    context_rewards = np.zeros((num_envs, horizon, 1))
    cum_means = []
    for h in range(horizon):
        batch = {"context_states": context_states[:, :h, :], "context_actions": context_actions[:, :h, :],
                 "context_next_states": context_next_states[:, :h, :], "context_rewards": context_rewards[:, :h, :]}
        controller.set_batch_numpy_vec(batch)
        states_lnr, actions_lnr, next_states_lnr, rewards_lnr = vec_env.deploy(controller)
        context_states[:, h, :] = states_lnr
        context_actions[:, h, :] = actions_lnr
        context_next_states[:, h, :] = next_states_lnr
        context_rewards[:, h, :] = rewards_lnr[:, None]
        cum_means.append(vec_env.get_arm_value(actions_lnr))
    cum_means = np.array(cum_means)
    if not include_meta:
        return cum_means
    return cum_means, {"context_states": context_states, "context_actions": context_actions,
                       "context_next_states": context_next_states, "context_rewards": context_rewards}


def regret_stats(all_means):
    """Suboptimality and cumulative-regret mean / SEM over tasks (evals/eval_bandit.py:169-178)."""
    import scipy.stats
    all_means = {k: np.array(v) for k, v in all_means.items()}
    diff = {k: all_means["opt"] - v for k, v in all_means.items()}
    cr = {k: np.cumsum(v, axis=1) for k, v in diff.items()}
    return dict(means={k: np.mean(v, axis=0) for k, v in diff.items()},
                sems={k: scipy.stats.sem(v, axis=0) for k, v in diff.items()},
                regret_means={k: np.mean(v, axis=0) for k, v in cr.items()},
                regret_sems={k: scipy.stats.sem(v, axis=0) for k, v in cr.items()})


def _baselines(envs, var, kind):
    """Classical comparison policies (ctrls/ctrl_bandit.py:57-380), when built."""
    try:
        from ctrls import ctrl_bandit as cb
    except ImportError:  # pragma: no cover
        return []
    out = []
    n = len(envs)
    if kind == "online":
        if hasattr(cb, "EmpMeanPolicy"):
            out.append(("Emp", cb.EmpMeanPolicy(envs[0], online=True, batch_size=n)))
        if hasattr(cb, "UCBPolicy"):
            out.append(("UCB1.0", cb.UCBPolicy(envs[0], const=1.0, batch_size=n)))
        if hasattr(cb, "ThompsonSamplingPolicy"):
            out.append(("Thomp", cb.ThompsonSamplingPolicy(envs[0], std=var, sample=True, prior_mean=0.5,
                                                             prior_var=1 / 12.0, warm_start=False, batch_size=n)))
    return out


def online(eval_trajs, model, n_eval, horizon, var, bandit_type):
    """Online regret of Opt vs the DPT learner (+ built baselines) (evals/eval_bandit.py:107-211)."""
    import matplotlib.pyplot as plt
    envs = [BanditEnv(eval_trajs[i]["means"], horizon, var=var) for i in range(n_eval)]
    vec_env = BanditEnvVec(envs)
    all_means = {}
    all_means["opt"] = deploy_online_vec(vec_env, OptPolicy(envs, batch_size=len(envs)), horizon).T
    ctrl = BanditTransformerController(model, sample=True, batch_size=len(envs))
    all_means["Lnr"] = deploy_online_vec(vec_env, ctrl, horizon).T
    for name, c in _baselines(envs, var, "online"):
        all_means[name] = deploy_online_vec(vec_env, c, horizon).T
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


def offline(eval_trajs, model, n_eval, horizon, var, bandit_type):
    """Offline evaluation on a fixed context, var forced to 0 (evals/eval_bandit.py:214-301)."""
    import matplotlib.pyplot as plt
    num_envs = len(eval_trajs)
    tmp_env = BanditEnv(eval_trajs[0]["means"], horizon, var=var)
    cs = np.zeros((num_envs, horizon, tmp_env.dx))
    ca = np.zeros((num_envs, horizon, tmp_env.du))
    cn = np.zeros((num_envs, horizon, tmp_env.dx))
    cr = np.zeros((num_envs, horizon, 1))
    envs = []
    for i in range(n_eval):
        traj = eval_trajs[i]
        envs.append(BanditEnv(traj["means"], horizon, var=var))
        cs[i] = traj["context_states"][:horizon]
        ca[i] = traj["context_actions"][:horizon]
        cn[i] = traj["context_next_states"][:horizon]
        cr[i] = traj["context_rewards"][:horizon, None]
    vec_env = BanditEnvVec(envs)
    batch = {"context_states": cs[:n_eval], "context_actions": ca[:n_eval], "context_next_states": cn[:n_eval],
             "context_rewards": cr[:n_eval]}
    opt_policy = OptPolicy(envs, batch_size=n_eval)
    lnr_policy = BanditTransformerController(model, sample=False, batch_size=n_eval)
    opt_policy.set_batch_numpy_vec(batch)
    lnr_policy.set_batch_numpy_vec(batch)
    _, _, _, rs_opt = vec_env.deploy_eval(opt_policy)
    _, _, _, rs_lnr = vec_env.deploy_eval(lnr_policy)
    baselines = {"opt": np.array(rs_opt), "lnr": np.array(rs_lnr)}
    for name, cls in (("emp", "EmpMeanPolicy"), ("thmp", "ThompsonSamplingPolicy"), ("lcb", "PessMeanPolicy")):
        from ctrls import ctrl_bandit as cb
        if hasattr(cb, cls):
            if cls == "EmpMeanPolicy":
                pol = cb.EmpMeanPolicy(envs[0], online=False, batch_size=n_eval)
            elif cls == "ThompsonSamplingPolicy":
                pol = cb.ThompsonSamplingPolicy(envs[0], std=var, sample=False, prior_mean=0.5, prior_var=1 / 12.0,
                                                warm_start=False, batch_size=n_eval)
            else:
                pol = cb.PessMeanPolicy(envs[0], const=0.8, batch_size=n_eval)
            pol.set_batch_numpy_vec(batch)
            baselines[name] = np.array(vec_env.deploy_eval(pol)[3])
    means = {k: np.mean(v) for k, v in baselines.items()}
    colors = plt.cm.viridis(np.linspace(0, 1, len(means)))
    plt.bar(means.keys(), means.values(), color=colors)
    plt.title(f"Mean Reward on {n_eval} Trajectories")
    return baselines


def offline_graph(eval_trajs, model, n_eval, horizon, var, bandit_type):
    """Offline suboptimality vs dataset size at 50 context lengths (evals/eval_bandit.py:304-335)."""
    import matplotlib.pyplot as plt
    import scipy.stats
    horizons = np.linspace(1, horizon, 50, dtype=int)
    all_means = []
    for h in horizons:
        baselines = offline(eval_trajs, model, n_eval=n_eval, horizon=h, var=var, bandit_type=bandit_type)
        plt.clf()
        means = {k: np.mean(v, axis=0) for k, v in baselines.items()}
        sems = {k: scipy.stats.sem(v, axis=0) for k, v in baselines.items()}
        all_means.append(means)
    for key in means.keys():
        if key != "opt":
            regrets = np.array([all_means[i]["opt"] - all_means[i][key] for i in range(len(horizons))])
            plt.plot(horizons, regrets, label=key)
            plt.fill_between(horizons, regrets - sems[key], regrets + sems[key], alpha=0.2)
    plt.legend()
    plt.yscale("log")
    plt.xlabel("Dataset size")
    plt.ylabel("Suboptimality")
    return horizons, all_means
