"""Dataset collection — drop-in for the reference collect_data.py (same CLI, same
pickled ``list[dict]`` trajectory format and filenames).

Every rollin of every task runs in ONE kernel launch (dpt_rollin_bandit /
dpt_rollin_darkroom) instead of a Python loop over envs x steps.  Task
sampling and the per-rollin behaviour policy (cov pick, Dirichlet draw,
random arm: collect_data.py:30-36) stay numpy draws on the host, vectorised.
"""
import argparse
import os
import pickle
import random

import numpy as np

import common_args
import dpt_hip
from envs import bandit_env, darkroom_env
from utils import build_bandit_data_filename, build_darkroom_data_filename, build_linear_bandit_data_filename

COV_CHOICES = np.array([0.0, .1, .2, .3, .4, .5, .6, .7, .8, .9, 1.0])


def behaviour_policies(M, A):
    """Per-rollin behaviour policy p = (1-cov) Dir(1_A) + cov e_rand (collect_data.py:30-36);
    the reference ignores the ``cov`` argument here and draws it from the 11-point grid."""
    cov = COV_CHOICES[np.random.randint(0, len(COV_CHOICES), M)]
    probs = np.random.dirichlet(np.ones(A), M)
    rand_index = np.random.randint(0, A, M)
    probs2 = np.zeros((M, A))
    probs2[np.arange(M), rand_index] = 1.0
    return (1 - cov)[:, None] * probs + cov[:, None] * probs2


def _bandit_rollins(means, H, var, type_code, probs):
    """Device rollins for M tasks -> (xs, us, xps, rs) numpy arrays with the reference dtypes."""
    acts, rews = dpt_hip.rollin_bandit(means, probs, H, var, type_code, seed=dpt_hip.next_seed())
    acts = acts.cpu().numpy()
    A = means.shape[1]
    M = len(acts)
    ones = np.ones((M, H, 1), dtype=np.int64)
    return ones, np.eye(A)[acts], ones.copy(), rews.cpu().numpy()


def rollin_bandit(env, cov, orig=False):
    """collect_data.py:23-53 for one env (the batched form is used by the generators)."""
    probs = behaviour_policies(1, env.dim)
    xs, us, xps, rs = _bandit_rollins(np.asarray(env.means, np.float64)[None], env.H_context, env.var,
                                      dpt_hip.BANDIT_GAUSSIAN if env.type == "uniform" else dpt_hip.BANDIT_BERNOULLI,
                                      probs)
    return xs[0], us[0], xps[0], rs[0]


def rollin_linear_bandit_vec(envs, noise=None, policy_noise=None):
    """collect_data.py:56-80: Thompson-sampling rollout (prior N(0, 1)) through deploy_online_vec.
    ``noise`` (H, N) reward normals and ``policy_noise`` (H, N, A) posterior normals, optional:
    the reference's np.random.normal draws, injected (default: Philox)."""
    from ctrls.ctrl_bandit import ThompsonSamplingPolicy
    from evals import eval_bandit
    H = envs[0].H_context
    thmp = ThompsonSamplingPolicy(envs[0], std=envs[0].var, sample=True, prior_mean=0.0, prior_var=1.0,
                                  warm_start=False, batch_size=len(envs))
    vec_env = bandit_env.BanditEnvVec(envs)
    _, meta = eval_bandit.deploy_online_vec(vec_env, thmp, H, include_meta=True, noise=noise,
                                            policy_noise=policy_noise)
    return (meta["context_states"], meta["context_actions"], meta["context_next_states"],
            meta["context_rewards"][:, :, 0])


def rollin_mdp(env, rollin_type):
    """collect_data.py:83-111 for one env."""
    out = _mdp_rollins([env], env.horizon, rollin_type)
    return out[0][0], out[1][0], out[2][0], out[3][0]


def _mdp_rollins(envs, H, rollin_type):
    mode = {"uniform": 0, "expert": 1}.get(rollin_type)
    if mode is None:
        raise NotImplementedError
    goals = np.stack([np.asarray(e.goal, np.int32) for e in envs])
    perm = None
    if any(getattr(e, "perm", None) is not None for e in envs):
        perm = np.stack([np.asarray(e.perm if e.perm is not None else range(5), np.int32) for e in envs])
    o = dpt_hip.rollin_darkroom(goals, H, envs[0].dim, perm, mode, seed=dpt_hip.next_seed())
    s = o["states"].cpu().numpy().astype(np.int64)
    a = np.eye(5)[o["actions"].cpu().numpy()]
    ns = o["next_states"].cpu().numpy().astype(np.int64)
    r = o["rewards"].cpu().numpy().astype(np.int64)
    return s, a, ns, r


def generate_bandit_histories_from_envs(envs, n_hists, n_samples, cov, type):
    """collect_data.py:158-182: n_hists rollins per env, each shared by n_samples trajectories."""
    M = len(envs) * n_hists
    A = envs[0].dim
    means = np.repeat(np.stack([np.asarray(e.means, np.float64) for e in envs]), n_hists, axis=0)
    probs = behaviour_policies(M, A)
    code = dpt_hip.BANDIT_GAUSSIAN if type == "uniform" else dpt_hip.BANDIT_BERNOULLI
    xs, us, xps, rs = _bandit_rollins(means, envs[0].H_context, envs[0].var, code, probs)
    trajs = []
    for e_i, env in enumerate(envs):
        for j in range(n_hists):
            m = e_i * n_hists + j
            for _ in range(n_samples):
                trajs.append({"query_state": np.array([1]), "optimal_action": env.opt_a,
                              "context_states": xs[m], "context_actions": us[m], "context_next_states": xps[m],
                              "context_rewards": rs[m], "means": env.means})
    return trajs


def generate_mdp_histories_from_envs(envs, n_hists, n_samples, rollin_type):
    """collect_data.py:189-218: rollins + per-sample query state and expert label."""
    rep = [env for env in envs for _ in range(n_hists)]
    s, a, ns, r = _mdp_rollins(rep, envs[0].horizon, rollin_type)
    M = len(rep)
    q = np.random.randint(0, envs[0].dim, (M, n_samples, 2))
    goals = np.repeat(np.stack([np.asarray(e.goal, np.int32) for e in rep]), n_samples, axis=0)
    perm = None
    if any(getattr(e, "perm", None) is not None for e in rep):
        perm = np.repeat(np.stack([np.asarray(e.perm if e.perm is not None else range(5), np.int32) for e in rep]),
                         n_samples, axis=0)
    opt = dpt_hip.darkroom_opt_action(q.reshape(-1, 2), goals, perm).cpu().numpy().reshape(M, n_samples)
    trajs = []
    for m, env in enumerate(rep):
        for k in range(n_samples):
            t = {"query_state": q[m, k].astype(np.int64), "optimal_action": np.eye(5)[opt[m, k]],
                 "context_states": s[m], "context_actions": a[m], "context_next_states": ns[m],
                 "context_rewards": r[m], "goal": env.goal}
            if hasattr(env, "perm_index"):
                t["perm_index"] = env.perm_index
            trajs.append(t)
    return trajs


def generate_bandit_histories(n_envs, dim, horizon, var, **kwargs):
    envs = [bandit_env.sample(dim, horizon, var) for _ in range(n_envs)]
    return generate_bandit_histories_from_envs(envs, **kwargs)


def generate_linear_bandit_histories(n_envs, dim, lin_d, horizon, var, **kwargs):
    """collect_data.py:228-284 (reads n_hists from kwargs; the reference reads a module global)."""
    rng = np.random.RandomState(seed=1234)
    arms = rng.normal(size=(dim, lin_d)) / np.sqrt(lin_d)
    envs = [bandit_env.sample_linear(arms, horizon, var) for _ in range(n_envs)]
    data_type = kwargs["data_type"]
    n_hists, n_samples = kwargs["n_hists"], kwargs["n_samples"]
    if data_type == "thompson":
        rolls = [rollin_linear_bandit_vec(envs) for _ in range(n_hists)]
        stacked = [np.stack([r[i] for r in rolls], axis=1) for i in range(4)]
    elif data_type == "uniform":
        M = len(envs) * n_hists
        means = np.repeat(np.stack([e.means for e in envs]), n_hists, axis=0)
        probs = np.zeros((M, dim))
        probs += behaviour_policies(M, dim)  # cov redrawn inside, as rollin_bandit does
        xs, us, xps, rs = _bandit_rollins(means, horizon, var, dpt_hip.BANDIT_GAUSSIAN, probs)
        stacked = [x.reshape(len(envs), n_hists, *x.shape[1:]) for x in (xs, us, xps, rs)]
    else:
        raise ValueError("Invalid data type")
    trajs = []
    for i, env in enumerate(envs):
        for j in range(n_hists):
            for _ in range(n_samples):
                trajs.append({"query_state": np.array([1]), "optimal_action": env.opt_a,
                              "context_states": stacked[0][i, j], "context_actions": stacked[1][i, j],
                              "context_next_states": stacked[2][i, j], "context_rewards": stacked[3][i, j],
                              "means": env.means, "arms": arms, "theta": env.theta, "var": env.var})
    return trajs


def generate_darkroom_histories(goals, dim, horizon, **kwargs):
    envs = [darkroom_env.DarkroomEnv(dim, goal, horizon) for goal in goals]
    return generate_mdp_histories_from_envs(envs, **kwargs)


def generate_darkroom_permuted_histories(indices, dim, horizon, **kwargs):
    envs = [darkroom_env.DarkroomEnvPermuted(dim, index, horizon) for index in indices]
    return generate_mdp_histories_from_envs(envs, **kwargs)


def main(argv=None):
    np.random.seed(0)
    random.seed(0)
    parser = argparse.ArgumentParser()
    common_args.add_dataset_args(parser)
    args = vars(parser.parse_args(argv))
    print("Args: ", args)
    env = args["env"]
    n_envs, n_eval_envs = args["envs"], args["envs_eval"]
    horizon, dim, var, cov, lin_d = args["H"], args["dim"], args["var"], args["cov"], args["lin_d"]
    n_train_envs = int(.8 * n_envs)
    n_test_envs = n_envs - n_train_envs
    config = {"n_hists": args["hists"], "n_samples": args["samples"], "horizon": horizon}

    if env == "bandit":
        config.update({"dim": dim, "var": var, "cov": cov, "type": "uniform"})
        train = generate_bandit_histories(n_train_envs, **config)
        test = generate_bandit_histories(n_test_envs, **config)
        evals = generate_bandit_histories(n_eval_envs, **config)
        paths = [build_bandit_data_filename(env, n_envs, config, mode=0),
                 build_bandit_data_filename(env, n_envs, config, mode=1),
                 build_bandit_data_filename(env, n_eval_envs, config, mode=2)]
    elif env == "linear_bandit":
        config.update({"dim": dim, "lin_d": lin_d, "var": var, "cov": cov, "data_type": "thompson"})
        train = generate_linear_bandit_histories(n_train_envs, **config)
        test = generate_linear_bandit_histories(n_test_envs, **config)
        evals = generate_linear_bandit_histories(n_eval_envs, **config)
        paths = [build_linear_bandit_data_filename(env, n_envs, config, mode=0),
                 build_linear_bandit_data_filename(env, n_envs, config, mode=1),
                 build_linear_bandit_data_filename(env, n_eval_envs, config, mode=2)]
    elif env == "darkroom_heldout":
        config.update({"dim": dim, "rollin_type": "uniform"})
        goals = np.array([[(j, i) for i in range(dim)] for j in range(dim)]).reshape(-1, 2)
        np.random.RandomState(seed=0).shuffle(goals)
        split = int(.8 * len(goals))
        train_goals, test_goals = goals[:split], goals[split:]
        eval_goals = np.array(test_goals.tolist() * int(100 // len(test_goals)))
        train_goals = np.repeat(train_goals, n_envs // (dim * dim), axis=0)
        test_goals = np.repeat(test_goals, n_envs // (dim * dim), axis=0)
        train = generate_darkroom_histories(train_goals, **config)
        test = generate_darkroom_histories(test_goals, **config)
        evals = generate_darkroom_histories(eval_goals, **config)
        paths = [build_darkroom_data_filename(env, n_envs, config, mode=0),
                 build_darkroom_data_filename(env, n_envs, config, mode=1),
                 build_darkroom_data_filename(env, 100, config, mode=2)]
    else:
        # miniworld needs a 3-D renderer (out of scope); darkroom_permuted is unwired in the reference too
        raise NotImplementedError

    os.makedirs("datasets", exist_ok=True)
    for path, data in zip(paths, (train, test, evals)):
        with open(path, "wb") as f:
            pickle.dump(data, f)
        print(f"Saved to {path}.")


if __name__ == "__main__":
    main()
