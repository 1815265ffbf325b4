"""Generate the golden fixtures under tests/golden/ by running the REFERENCE.

Test infrastructure only.  This script imports the read-only reference checkout
(``/root/reference``, titanium-47/decision-pretrained-transformer) on CPU and
records inputs + outputs of the hot-path functions as small ``.npz`` files.
The reference never travels with the repo: only these vectors do.

Randomness is captured, not re-implemented: every ``np.random.choice`` /
``np.random.normal`` call the reference makes is wrapped; before the real call
a replica ``RandomState`` is built from the global state and asked for the one
``random_sample()`` / ``standard_normal()`` draw the call consumes.  After the
real call the replica and the global state are asserted identical, which proves
the recorded draw is exactly what the reference used.  This pins the two
algebraic identities the device path relies on:

* ``np.random.choice(A, p=p) == searchsorted(cumsum(p64)/cumsum(p64)[-1], u, 'right')``
  (numpy legacy ``RandomState.choice``, numpy 2.2.6 — not vendored in the reference),
* ``np.random.normal(0, s) == 0.0 + s * g`` with ``g = standard_normal()``.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py
The script refuses to run when /root/reference is absent (GPU box).
"""
import os
import sys
import types

sys.dont_write_bytecode = True  # never leave __pycache__ in the reference tree

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    """Minimal stand-ins for modules the reference imports but never computes with.

    gym: only ``gym.Env`` (base class) and ``gym.spaces.Box/Discrete`` (attribute
    holders) are touched (envs/base_env.py:8, envs/bandit_env.py:37-38,
    envs/darkroom_env.py:19-21).  IPython: ``embed`` is imported, never called.
    skimage: ``resize`` is imported at collect_data.py:8 for Miniworld only.
    """
    gym = types.ModuleType("gym")

    class Env:  # noqa: D401
        pass

    class Box:
        def __init__(self, low=None, high=None, shape=None):
            self.low, self.high, self.shape = low, high, shape

    class Discrete:
        def __init__(self, n):
            self.n = n

    gym.Env = Env
    gym.spaces = types.SimpleNamespace(Box=Box, Discrete=Discrete)
    sys.modules["gym"] = gym
    ipy = types.ModuleType("IPython")
    ipy.embed = lambda *a, **k: None
    ipy.get_ipython = lambda: None
    ipy.version_info = (9, 0, 0)  # matplotlib's backend check returns early for >= 8.24
    sys.modules["IPython"] = ipy
    sk = types.ModuleType("skimage")
    skt = types.ModuleType("skimage.transform")
    skt.resize = lambda *a, **k: None
    sk.transform = skt
    sys.modules["skimage"] = sk
    sys.modules["skimage.transform"] = skt


class DrawRecorder:
    """Wraps np.random.choice / np.random.normal and records the consumed draws."""

    def __init__(self, np):
        self.np = np
        self.u = []
        self.g = []
        self.choice_kind = []
        self.plain = []
        self.garr = []
        self._choice = np.random.choice
        self._normal = np.random.normal

    def _replica(self):
        rs = self.np.random.RandomState()
        rs.set_state(self.np.random.get_state())
        return rs

    def _same_state(self, rs):
        a = self.np.random.get_state()
        b = rs.get_state()
        return (a[0] == b[0] and (a[1] == b[1]).all() and a[2] == b[2]
                and a[3] == b[3] and a[4] == b[4])

    def choice(self, a, size=None, replace=True, p=None):
        np = self.np
        if p is not None and size is None:
            rs = self._replica()
            u = rs.random_sample()
            out = self._choice(a, size=size, replace=replace, p=p)
            assert self._same_state(rs), "choice consumed != one uniform"
            p64 = np.asarray(p, dtype=np.float64)
            cdf = p64.cumsum()
            cdf /= cdf[-1]
            idx = int(cdf.searchsorted(u, side="right"))
            assert np.asarray(a)[idx] == out, "choice != searchsorted(cdf,u)"
            self.u.append(u)
            self.choice_kind.append(1)
            return out
        out = self._choice(a, size=size, replace=replace, p=p)
        self.choice_kind.append(0)
        self.plain.append(out)
        return out

    def normal(self, loc=0.0, scale=1.0, size=None):
        np = self.np
        if size is None and np.ndim(loc) == 0 and np.ndim(scale) == 0:
            rs = self._replica()
            g = rs.standard_normal()
            out = self._normal(loc, scale)
            assert self._same_state(rs), "normal consumed != one gaussian"
            assert out == loc + scale * g, "normal(loc,s) != loc + s*g"
            self.g.append(g)
            return out
        if size is None:  # array loc/scale (Thompson posterior draw, ctrl_bandit.py:232)
            rs = self._replica()
            g = rs.standard_normal(np.broadcast(loc, scale).shape)
            out = self._normal(loc, scale)
            assert self._same_state(rs), "array normal consumed != standard_normal(shape)"
            assert np.array_equal(out, loc + scale * g), "normal(loc,s) != loc + s*g (array)"
            self.garr.append(g)
            return out
        return self._normal(loc, scale, size)

    def __enter__(self):
        self.np.random.choice = self.choice
        self.np.random.normal = self.normal
        return self

    def __exit__(self, *exc):
        self.np.random.choice = self._choice
        self.np.random.normal = self._normal


def perturbed_state_dict(model, seed, scale=0.05):
    """Reference init (GPT2 scheme) + seeded N(0,1)*scale perturbation so every
    parameter (LN gains/biases included) carries signal."""
    import numpy as np
    import torch
    rs = np.random.RandomState(seed)
    sd = model.state_dict()
    for k in sorted(sd.keys()):
        v = sd[k]
        if k.endswith("wte.weight") or not v.dtype.is_floating_point:
            continue
        noise = torch.from_numpy(rs.standard_normal(tuple(v.shape)).astype(np.float32))
        sd[k] = v + scale * noise
    model.load_state_dict(sd)
    return {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()
            if not k.endswith("wte.weight")}


def baselines():
    """F8: the classical policies of eval_bandit.online / offline, through the reference loop."""
    import numpy as np
    from envs import bandit_env
    from ctrls import ctrl_bandit as cb
    from evals import eval_bandit, eval_linear_bandit

    def run(mod, envs, ctrl, H, seed):
        vec = bandit_env.BanditEnvVec(envs)
        np.random.seed(seed)
        with DrawRecorder(np) as rec:
            cm, meta = mod.deploy_online_vec(vec, ctrl, H, include_meta=True)
        return cm, meta, rec

    out = {}
    rs = np.random.RandomState(81)
    N, H, A, var = 200, 24, 5, 0.3  # UCBPolicy.act_numpy_vec only works for 200 tasks (ctrl_bandit.py:374)
    means = rs.uniform(0, 1, (N, A))
    out["means"] = means
    for name, mk in (("emp", lambda e: cb.EmpMeanPolicy(e[0], online=True, batch_size=N)),
                     ("ucb", lambda e: cb.UCBPolicy(e[0], const=1.0, batch_size=N)),
                     ("thomp", lambda e: cb.ThompsonSamplingPolicy(e[0], std=var, sample=True, prior_mean=0.5,
                                                                     prior_var=1 / 12.0, warm_start=False,
                                                                     batch_size=N))):
        envs = [bandit_env.BanditEnv(m, H, var=var) for m in means]
        cm, meta, rec = run(eval_bandit, envs, mk(envs), H, 90 + len(name))
        out[f"{name}/cum_means"] = cm
        out[f"{name}/actions"] = meta["context_actions"].argmax(-1)
        out[f"{name}/rewards"] = meta["context_rewards"][..., 0]
        out[f"{name}/g"] = np.array(rec.g).reshape(H, N)
        if rec.garr:
            out[f"{name}/policy_g"] = np.stack(rec.garr)  # (H, N, A)
    # offline decisions on a fixed context (var forced to 0 by deploy_eval)
    h = 30
    ca = np.eye(A)[rs.randint(0, A, (N, h))]
    cr = (means[np.arange(N)[:, None], ca.argmax(-1)] + 0.3 * rs.normal(size=(N, h)))[..., None]
    batch = {"context_states": np.ones((N, h, 1)), "context_actions": ca, "context_next_states": np.ones((N, h, 1)),
             "context_rewards": cr}
    out.update({"off/ctx_actions": ca.argmax(-1), "off/ctx_rewards": cr[..., 0]})
    envs = [bandit_env.BanditEnv(m, h, var=var) for m in means]
    vec = bandit_env.BanditEnvVec(envs)
    for name, pol in (("emp", cb.EmpMeanPolicy(envs[0], online=False, batch_size=N)),
                      ("lcb", cb.PessMeanPolicy(envs[0], const=.8, batch_size=N))):
        pol.set_batch_numpy_vec(batch)
        _, us, _, rsum = vec.deploy_eval(pol)
        out[f"off/{name}/actions"] = us.argmax(-1)
        out[f"off/{name}/rewards"] = rsum
    # LinUCB on linear bandits (eval_linear_bandit.online leg)
    arms = np.random.RandomState(1234).normal(size=(10, 2)) / np.sqrt(2)
    thetas = rs.normal(0, 1, (N, 2)) / np.sqrt(2)
    lenvs = [bandit_env.LinearBanditEnv(t, arms, 16, var=var) for t in thetas]
    cm, meta, rec = run(eval_linear_bandit, lenvs, cb.LinUCBPolicy(lenvs[0], const=1.0, batch_size=N), 16, 77)
    out.update({"lin/means": np.stack([e.means for e in lenvs]), "lin/arms": arms, "lin/cum_means": cm,
                "lin/actions": meta["context_actions"].argmax(-1), "lin/g": np.array(rec.g).reshape(16, N),
                "lin/first_action": np.asarray(rec.plain[0])})
    np.savez_compressed(os.path.join(OUT, "baselines.npz"), **out)
    print("F8 baselines")


def host_surface():
    """F9: filenames (utils.py:14-190) and argparse defaults (common_args.py:2-59) -> JSON."""
    import argparse
    import json
    import utils
    import common_args
    cases = []
    cfgs = [dict(n_hists=1, n_samples=1, horizon=500, dim=5, var=0.3, cov=0.0, lin_d=2, rollin_type="uniform"),
            dict(n_hists=3, n_samples=2, horizon=100, dim=10, var=0.0, cov=0.5, lin_d=3, rollin_type="uniform")]
    for cfg in cfgs:
        for mode in (0, 1, 2):
            cases.append(["build_bandit_data_filename", ["bandit", 100000, cfg, mode],
                          utils.build_bandit_data_filename("bandit", 100000, cfg, mode)])
            cases.append(["build_linear_bandit_data_filename", ["linear_bandit", 1000, cfg, mode],
                          utils.build_linear_bandit_data_filename("linear_bandit", 1000, cfg, mode)])
            cases.append(["build_darkroom_data_filename", ["darkroom_heldout", 100, cfg, mode],
                          utils.build_darkroom_data_filename("darkroom_heldout", 100, cfg, mode)])
    mcfg = dict(shuffle=True, lr=0.0001, dropout=0, n_embd=32, n_layer=4, n_head=4, n_envs=100000, n_hists=1,
                n_samples=1, var=0.3, cov=0.0, horizon=500, dim=5, seed=1, lin_d=2)
    for fn, env in (("build_bandit_model_filename", "bandit"), ("build_linear_bandit_model_filename", "linear_bandit"),
                    ("build_darkroom_model_filename", "darkroom_heldout")):
        cases.append([fn, [env, mcfg], getattr(utils, fn)(env, mcfg)])
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_train_args(p)
    common_args.add_eval_args(p)
    defaults = vars(p.parse_args(["--env", "bandit"]))
    json.dump({"filenames": cases, "defaults": defaults}, open(os.path.join(OUT, "host_surface.json"), "w"),
              indent=1, sort_keys=True)
    print("F9 host_surface")


def fixture_transformer(name, horizon=None):
    """The reference Transformer (models/net.py:9-60) holding the weights recorded in
    forward_<name>.npz; a shorter ``horizon`` keeps the first 4(1+horizon) wpe rows (the
    model the reference builds for that horizon, with the same parameters)."""
    import numpy as np
    import torch
    from net import Transformer
    g = dict(np.load(os.path.join(OUT, f"forward_{name}.npz")))
    H, sd_, ad, L, E = (int(x) for x in g["cfg"])
    horizon = horizon or H
    m = Transformer(dict(horizon=horizon, state_dim=sd_, action_dim=ad, n_layer=L, n_embd=E, n_head=4,
                         dropout=0.0, test=True))
    state = m.state_dict()
    for k, v in g.items():
        if k.startswith("w/"):
            key = k[2:]
            if key.endswith("wpe.weight"):
                v = v[: 4 * (1 + horizon)]
            state[key] = torch.from_numpy(v)
    m.load_state_dict(state)
    m.eval()
    return m


def c1():
    """BASELINE config 1 at its size: 5-arm Gaussian bandit, H=100, 64 tasks, var 0.3 (run_bandit.sh
    flags).  (a) collect: generate_bandit_histories (collect_data.py:158-182, :221-225) with every
    draw recorded per env (cov pick, Dirichlet, random arm, the H arm choices and reward normals);
    (b) eval: the online deploy_online_vec loop (evals/eval_bandit.py:56-103) of the DPT sampling
    controller (model: forward_bandit5 weights at horizon 100) with its uniforms / normals, plus the
    Opt leg and the regret curves of evals/eval_bandit.py:169-178."""
    import numpy as np
    import scipy.stats
    import torch
    import collect_data
    from envs import bandit_env
    from ctrls.ctrl_bandit import BanditTransformerController, OptPolicy
    from evals import eval_bandit
    N, H, A, var = 64, 100, 5, 0.3
    out = {}
    np.random.seed(2024)
    rec_dir = []
    real_dir = np.random.dirichlet

    def dirichlet(alpha, _r=real_dir):
        v = _r(alpha)
        rec_dir.append(v)
        return v

    np.random.dirichlet = dirichlet
    try:
        with DrawRecorder(np) as rec:
            trajs = collect_data.generate_bandit_histories(N, dim=A, horizon=H, var=var, n_hists=1, n_samples=1,
                                                           cov=0.0, type="uniform")
    finally:
        np.random.dirichlet = real_dir
    # per env: uniform(0,1,A) means (bandit_env.sample: no recorded draw), then cov pick + random
    # arm (plain choices), H choice uniforms and H reward normals
    assert len(rec.plain) == 2 * N and len(rec.u) == N * H and len(rec.g) == N * H
    out["collect/means"] = np.stack([t["means"] for t in trajs])
    out["collect/cov"] = np.array(rec.plain[0::2], np.float64)
    out["collect/rand_index"] = np.array(rec.plain[1::2], np.int64)
    out["collect/dirichlet"] = np.stack(rec_dir)
    out["collect/u"] = np.array(rec.u).reshape(N, H)
    out["collect/g"] = np.array(rec.g).reshape(N, H)
    for t in trajs:  # the bandit state is the constant [1] (collect_data.py:41)
        assert (t["context_states"] == 1).all() and (t["context_next_states"] == 1).all()
        assert t["context_states"].shape == (H, 1) and t["context_states"].dtype == np.int64
    out["collect/actions"] = np.stack([t["context_actions"].argmax(-1) for t in trajs]).astype(np.int8)
    assert np.array_equal(np.eye(A)[out["collect/actions"]], np.stack([t["context_actions"] for t in trajs]))
    out["collect/rewards"] = np.stack([t["context_rewards"] for t in trajs])
    out["collect/optimal_action"] = np.stack([t["optimal_action"] for t in trajs])
    # online eval of the DPT policy on 64 fresh tasks
    means = np.random.RandomState(12).uniform(0, 1, (N, A))
    envs = [bandit_env.BanditEnv(m, H, var=var) for m in means]
    vec = bandit_env.BanditEnvVec(envs)
    model = fixture_transformer("bandit5", horizon=H)
    opt = eval_bandit.deploy_online_vec(vec, OptPolicy(envs, batch_size=N), H).T  # evals/eval_bandit.py:123-128
    ctrl = BanditTransformerController(model, sample=True, batch_size=N)
    np.random.seed(2025)
    with DrawRecorder(np) as rec, torch.no_grad():
        cm, meta = eval_bandit.deploy_online_vec(vec, ctrl, H, include_meta=True)
    assert (opt == means.max(1, keepdims=True)).all()  # the Opt leg: means[opt_a] every step
    out.update({"eval/means": means, "eval/cum_means": cm,
                "eval/actions": meta["context_actions"].argmax(-1), "eval/rewards": meta["context_rewards"][..., 0],
                "eval/u": np.array(rec.u).reshape(H, N), "eval/g": np.array(rec.g).reshape(H, N),
                "cfg": np.array([N, H, A]), "var": np.float64(var)})
    diff = opt - cm.T  # all_means_diff (evals/eval_bandit.py:169)
    cr = np.cumsum(diff, axis=1)
    out.update({"eval/subopt_mean": np.mean(diff, axis=0), "eval/subopt_sem": scipy.stats.sem(diff, axis=0),
                "eval/regret_mean": np.mean(cr, axis=0), "eval/regret_sem": scipy.stats.sem(cr, axis=0)})
    np.savez_compressed(os.path.join(OUT, "c1_bandit.npz"), **out)
    print("C1 collect + eval")


def gpu_bandit_env():
    """envs/gpu_bandit_env.py:53-74 on the CPU device with every torch.randn recorded: fp32 rewards
    mean_rewards + randn * var for 3 steps of 64 tasks at var 0.3 and 1.0, the done flags, the
    ValueError past H, and deploy_eval's var = 0 rewards."""
    import numpy as np
    import torch
    from envs.gpu_bandit_env import GPUBanditEnv
    out = {}
    real_randn = torch.randn
    for var in (0.3, 1.0):
        torch.manual_seed(int(var * 10))
        env = GPUBanditEnv(5, 64, 3, var=var, device=torch.device("cpu"))
        draws = []

        def randn(*a, _r=real_randn, **k):
            v = _r(*a, **k)
            draws.append(v.clone())
            return v

        torch.randn = randn
        try:
            env.reset()
            acts, rews, dones = [], [], []
            rs = np.random.RandomState(int(var * 10))
            for _ in range(3):
                us = torch.nn.functional.one_hot(torch.from_numpy(rs.randint(0, 5, 64)), 5).float()
                _, r, done, _ = env.step(us)
                acts.append(us.argmax(1).numpy())
                rews.append(r.numpy())
                dones.append(done.numpy())
            try:
                env.step(us)
                raise AssertionError("no ValueError past H")
            except ValueError as e:
                out[f"var{var}/error"] = np.array(str(e))
        finally:
            torch.randn = real_randn
        out.update({f"var{var}/means": env.means.numpy(), f"var{var}/actions": np.stack(acts),
                    f"var{var}/g": torch.stack(draws).numpy(), f"var{var}/rewards": np.stack(rews),
                    f"var{var}/done": np.stack(dones)})
    np.savez_compressed(os.path.join(OUT, "gpu_bandit_env.npz"), **out)
    print("GPUBanditEnv")


def linear_thompson():
    """collect_data.rollin_linear_bandit_vec (collect_data.py:56-80): the Thompson behaviour policy
    (prior mean 0, variance 1) on 10-arm linear bandits (lin_d = 2, arms RandomState(1234) as in
    collect_data.py:230-231) through deploy_online_vec, with the posterior normals and reward
    normals recorded."""
    import numpy as np
    import collect_data
    from envs import bandit_env
    N, H, A, d, var = 24, 30, 10, 2, 0.3
    arms = np.random.RandomState(1234).normal(size=(A, d)) / np.sqrt(d)
    thetas = np.random.RandomState(5).normal(0, 1, (N, d)) / np.sqrt(d)
    envs = [bandit_env.LinearBanditEnv(t, arms, H, var=var) for t in thetas]
    np.random.seed(77)
    with DrawRecorder(np) as rec:
        cs, ca, cn, cr = collect_data.rollin_linear_bandit_vec(envs)
    np.savez_compressed(os.path.join(OUT, "linear_thompson.npz"), arms=arms, theta=thetas,
                        means=np.stack([e.means for e in envs]), var=np.float64(var),
                        policy_g=np.stack(rec.garr), g=np.array(rec.g).reshape(H, N),
                        context_states=cs, context_actions=ca, context_next_states=cn, context_rewards=cr)
    print("linear Thompson rollin")


def darkroom_offline():
    """evals/eval_darkroom.py:124-189 (offline): the expert's return, the DPT sampled leg (its
    selection uniforms recorded) and the deterministic greedy leg on fixed contexts, plain and
    permuted; returns captured at DarkroomEnvVec.deploy_eval / DarkroomEnv.deploy_eval."""
    import numpy as np
    import torch
    import collect_data
    from envs import darkroom_env
    from evals import eval_darkroom
    model = fixture_transformer("darkroom")
    out = {}
    for tag, n, H, permuted in (("plain", 8, 30, False), ("permuted", 4, 20, True)):
        rs = np.random.RandomState(90 + n)
        np.random.seed(91 + n)
        trajs = []
        for i in range(n):
            if permuted:
                env = darkroom_env.DarkroomEnvPermuted(10, int(rs.randint(0, 120)), H)
            else:
                env = darkroom_env.DarkroomEnv(10, rs.randint(0, 10, 2), H)
            s, a, ns, r = collect_data.rollin_mdp(env, "uniform")  # collect_data.py:83-111
            t = {"context_states": s, "context_actions": a, "context_next_states": ns, "context_rewards": r,
                 "goal": env.goal}
            if permuted:
                t["perm_index"] = env.perm_index
            trajs.append(t)
        got = {"vec": [], "env": []}
        real_vec, real_env = darkroom_env.DarkroomEnvVec.deploy_eval, darkroom_env.DarkroomEnv.deploy_eval

        def vec_eval(self, ctrl, _r=real_vec):
            res = _r(self, ctrl)
            got["vec"].append(res[3])
            return res

        def env_eval(self, ctrl, _r=real_env):
            res = _r(self, ctrl)
            got["env"].append(res[3])
            return res

        darkroom_env.DarkroomEnvVec.deploy_eval = vec_eval
        darkroom_env.DarkroomEnv.deploy_eval = env_eval
        np.random.seed(93 + n)
        try:
            with DrawRecorder(np) as rec, torch.no_grad():
                eval_darkroom.offline(trajs, model, n_eval=n, H=H, dim=10, permuted=permuted)
        finally:
            darkroom_env.DarkroomEnvVec.deploy_eval, darkroom_env.DarkroomEnv.deploy_eval = real_vec, real_env
        assert len(got["vec"]) == 2 and len(got["env"]) == n and len(rec.u) == n * H
        for k in ("context_states", "context_actions", "context_next_states", "context_rewards", "goal"):
            out[f"{tag}/{k}"] = np.stack([t[k] for t in trajs])
        if permuted:
            out[f"{tag}/perm_index"] = np.array([t["perm_index"] for t in trajs])
        out.update({f"{tag}/opt_returns": np.array([np.sum(x) for x in got["env"]]),
                    f"{tag}/lnr_rewards": np.asarray(got["vec"][0]), f"{tag}/greedy_rewards": np.asarray(got["vec"][1]),
                    f"{tag}/u": np.array(rec.u).reshape(H, n), f"{tag}/cfg": np.array([n, H, int(permuted)])})
    np.savez_compressed(os.path.join(OUT, "darkroom_offline.npz"), **out)
    print("darkroom offline")


def train_grads():
    """train.py:286-331 on the reference model: preds = model(batch) with test=False
    (models/net.py:56-60, positions 1..T-1), CrossEntropyLoss(reduction='sum') against the optimal
    action repeated over the positions, loss.backward().  Recorded: loss, preds and every
    parameter's gradient, in fp32 (the reference as it runs) and with the same model in float64
    (the truth the fp32 results are measured against).  Two models: DarkRoom (sd 2, A 5) with a
    30-transition context, and the 5-arm bandit one with 20."""
    import numpy as np
    import torch
    out = {}
    for name, C, B in (("darkroom", 30, 4), ("bandit5", 20, 3)):
        rs = np.random.RandomState(300 + C)
        model = fixture_transformer(name)
        sd_, ad = model.config["state_dim"], model.config["action_dim"]
        if name == "darkroom":
            batch = {"query_states": rs.randint(0, 10, (B, sd_)), "context_states": rs.randint(0, 10, (B, C, sd_)),
                     "context_actions": np.eye(ad)[rs.randint(0, ad, (B, C))],
                     "context_next_states": rs.randint(0, 10, (B, C, sd_)),
                     "context_rewards": (rs.uniform(size=(B, C, 1)) < 0.2)}
        else:
            batch = {"query_states": np.ones((B, 1)), "context_states": np.ones((B, C, 1)),
                     "context_actions": np.eye(ad)[rs.randint(0, ad, (B, C))],
                     "context_next_states": np.ones((B, C, 1)), "context_rewards": rs.normal(0.5, 0.5, (B, C, 1))}
        batch = {k: np.asarray(v, np.float64) for k, v in batch.items()}
        batch["zeros"] = np.zeros((B, sd_ ** 2 + ad + 1))
        opt = np.eye(ad)[rs.randint(0, ad, B)]
        for k, v in batch.items():
            out[f"{name}/{k}"] = v
        out[f"{name}/optimal_actions"] = opt
        for tag, dt in (("f32", torch.float32), ("f64", torch.float64)):
            m = model.to(dt)
            m.test = False
            m.train()
            m.zero_grad()
            tb = {k: torch.tensor(v, dtype=dt) for k, v in batch.items()}
            pred = m(tb)                                             # train.py:302
            true = torch.tensor(opt, dtype=dt).unsqueeze(1).repeat(1, pred.shape[1], 1)
            loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, ad), true.reshape(-1, ad))
            loss.backward()                                          # train.py:309
            out[f"{name}/{tag}/loss"] = np.float64(loss.item())
            out[f"{name}/{tag}/preds"] = pred.detach().numpy()
            for k, p in m.named_parameters():
                if p.grad is not None and not k.endswith("wte.weight"):
                    gv = p.grad.detach().numpy()
                    if k.endswith("wpe.weight"):  # rows >= T get no gradient: keep the first T
                        assert not gv[C + 1:].any()
                        gv = gv[:C + 1]
                    out[f"{name}/{tag}/grad/{k}"] = gv
        # keep the float64 gradients; of the fp32 run only its error against them (per parameter,
        # relative to the largest float64 entry), the scale a fp32 implementation is held to
        for k in [k for k in out if k.startswith(f"{name}/f32/grad/")]:
            ref = out[k.replace("/f32/", "/f64/")]
            out[k.replace("/grad/", "/grad_err/")] = np.float64(np.abs(out.pop(k) - ref).max() / np.abs(ref).max())
        model.float()
    np.savez_compressed(os.path.join(OUT, "train_grads.npz"), **out)
    print("train grads")


def train_dropout():
    """train.py:286-331 with --dropout > 0: the reference model built with dropout p (GPT2Config
    embd/attn/resid_pdrop, models/net.py:30-32) in training mode, its every dropout call fed the
    mask the HIP kernels draw (include/dpt_hip.h dpt_train_desc: Philox(seed, (site, e / 4,
    DPT_STREAM_DROPOUT)) word e % 4 >= ceil(p 2^32), kept elements times float32(1 / (1 - p))).
    torch.nn.functional.dropout is replaced for the call and each call's site is checked by order
    and shape: 0 the embedding sum, then per layer the attention probabilities, c_proj's output
    and mlp.c_proj's output -- this pins WHERE GPT-2 drops, which is what the restatement must
    match (torch's own mask stream is not reproducible on the device, and is not the point).
    Attention runs "eager" for the recording: sdpa draws its probability mask inside the fused
    op, where no mask can be injected; eager applies the same dropout to the same softmax
    probabilities.  Float64, the bandit5 weights, two (p, seed) pairs."""
    import numpy as np
    import torch
    sys.path.insert(0, os.path.dirname(OUT))
    from philox_np import philox
    from net import Transformer
    g = dict(np.load(os.path.join(OUT, "forward_bandit5.npz")))
    H, sd_, ad, L, E = (int(x) for x in g["cfg"])
    C, B = 20, 3
    out = {}
    real = torch.nn.functional.dropout
    for case, (p, seed) in enumerate(((0.1, 77), (0.3, 2 ** 40 + 5))):
        m = Transformer(dict(horizon=H, state_dim=sd_, action_dim=ad, n_layer=L, n_embd=E, n_head=4, dropout=p,
                             test=False))
        state = m.state_dict()
        for k, v in g.items():
            if k.startswith("w/"):
                state[k[2:]] = torch.from_numpy(v)
        m.load_state_dict(state)
        m.transformer.set_attn_implementation("eager")
        m = m.double()
        m.train()
        rs = np.random.RandomState(900 + case)
        batch = {"query_states": np.ones((B, 1)), "context_states": np.ones((B, C, 1)),
                 "context_actions": np.eye(ad)[rs.randint(0, ad, (B, C))],
                 "context_next_states": np.ones((B, C, 1)), "context_rewards": rs.normal(0.5, 0.5, (B, C, 1))}
        batch["zeros"] = np.zeros((B, sd_ ** 2 + ad + 1))
        opt = np.eye(ad)[rs.randint(0, ad, B)]
        p32 = np.float32(p)
        thr = min(int(np.ceil(np.float64(p32) * 2.0 ** 32)), 2 ** 32 - 1)
        scale = np.float64(np.float32(1.0) / (np.float32(1.0) - p32))
        T = C + 1
        shapes = [(B, T, E)]
        for _ in range(L):
            shapes += [(B, 1, T, T), (B, T, E), (B, T, E)]
        calls = []

        def fake(x, p=0.5, training=True, inplace=False, _p=p):
            p_, p = p, _p
            site = len(calls)
            assert training and abs(p_ - p) < 1e-12, (site, p_, training)
            assert tuple(x.shape) == shapes[site], (site, tuple(x.shape), shapes[site])
            n = x.numel()
            w = np.stack(philox(seed, site, np.arange((n + 3) // 4), 3), 1).reshape(-1)[:n]
            k = torch.from_numpy(np.where(w >= thr, scale, 0.0).reshape(x.shape))
            calls.append(site)
            return x * k
        torch.nn.functional.dropout = fake
        try:
            tb = {k: torch.tensor(v, dtype=torch.float64) for k, v in batch.items()}
            m.zero_grad()
            pred = m(tb)                                             # train.py:302
            true = torch.tensor(opt, dtype=torch.float64).unsqueeze(1).repeat(1, pred.shape[1], 1)
            loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, ad), true.reshape(-1, ad))
            loss.backward()                                          # train.py:309
        finally:
            torch.nn.functional.dropout = real
        assert calls == list(range(len(shapes))), calls
        pre = f"c{case}/"
        for k, v in batch.items():
            out[pre + k] = np.asarray(v, np.float64)
        out[pre + "optimal_actions"] = opt
        out[pre + "p"] = np.float64(p)
        out[pre + "seed"] = np.uint64(seed)
        out[pre + "loss"] = np.float64(loss.item())
        out[pre + "preds"] = pred.detach().numpy()
        for k, prm in m.named_parameters():
            if prm.grad is not None and not k.endswith("wte.weight"):
                gv = prm.grad.detach().numpy()
                if k.endswith("wpe.weight"):
                    assert not gv[T:].any()
                    gv = gv[:T]
                out[pre + "grad/" + k] = gv
    np.savez_compressed(os.path.join(OUT, "train_dropout.npz"), **out)
    print("train dropout")


def linucb_d4():
    """LinUCB (ctrls/ctrl_bandit.py:447-528) on 12-arm linear bandits with lin_d = 4 (the --lin_d
    flag, common_args.py:15-16), through eval_linear_bandit.deploy_online_vec with every draw
    recorded (the random first arm, the reward normals)."""
    import numpy as np
    from envs import bandit_env
    from ctrls import ctrl_bandit as cb
    from evals import eval_linear_bandit
    N, H, A, d, var = 64, 20, 12, 4, 0.3
    arms = np.random.RandomState(1234).normal(size=(A, d)) / np.sqrt(d)   # collect_data.py:230-231
    thetas = np.random.RandomState(17).normal(0, 1, (N, d)) / np.sqrt(d)
    envs = [bandit_env.LinearBanditEnv(t, arms, H, var=var) for t in thetas]
    vec = bandit_env.BanditEnvVec(envs)
    np.random.seed(19)
    with DrawRecorder(np) as rec:
        cm, meta = eval_linear_bandit.deploy_online_vec(vec, cb.LinUCBPolicy(envs[0], const=1.0, batch_size=N), H,
                                                        include_meta=True)
    np.savez_compressed(os.path.join(OUT, "linucb_d4.npz"), means=np.stack([e.means for e in envs]), arms=arms,
                        theta=thetas,
                        cum_means=cm, actions=meta["context_actions"].argmax(-1), g=np.array(rec.g).reshape(H, N),
                        first_action=np.asarray(rec.plain[0]))
    print("LinUCB d=4")


def linucb_long():
    """LinUCB (ctrls/ctrl_bandit.py:447-528) with lin_d = 2 on the C4 arm table (20 arms,
    collect_data.py:230-231) over 800 steps, so the context crosses the BLAS blocking sizes
    (384 / 768 rows of the X^T X product): through eval_linear_bandit.deploy_online_vec with
    every draw recorded."""
    import numpy as np
    from envs import bandit_env
    from ctrls import ctrl_bandit as cb
    from evals import eval_linear_bandit
    N, H, A, d, var = 24, 800, 20, 2, 0.3
    arms = np.random.RandomState(1234).normal(size=(A, d)) / np.sqrt(d)
    thetas = np.random.RandomState(23).normal(0, 1, (N, d)) / np.sqrt(d)
    envs = [bandit_env.LinearBanditEnv(t, arms, H, var=var) for t in thetas]
    vec = bandit_env.BanditEnvVec(envs)
    np.random.seed(29)
    with DrawRecorder(np) as rec:
        cm, meta = eval_linear_bandit.deploy_online_vec(vec, cb.LinUCBPolicy(envs[0], const=1.0, batch_size=N), H,
                                                        include_meta=True)
    np.savez_compressed(os.path.join(OUT, "linucb_long.npz"), means=np.stack([e.means for e in envs]), arms=arms,
                        theta=thetas, cum_means=cm, actions=meta["context_actions"].argmax(-1).astype(np.int8),
                        g=np.array(rec.g).reshape(H, N), first_action=np.asarray(rec.plain[0]))
    print("LinUCB long")


def linucb_dims():
    """LinUCB (ctrls/ctrl_bandit.py:447-528) at lin_d 3, 5, 6 and 8 (every width the policy kernel
    takes besides 2 and 4, which linucb_long / linucb_d4 hold): 12-arm linear bandits over 100 steps
    through eval_linear_bandit.deploy_online_vec, every draw recorded."""
    import numpy as np
    from envs import bandit_env
    from ctrls import ctrl_bandit as cb
    from evals import eval_linear_bandit
    out = {}
    for d in (3, 5, 6, 8):
        N, H, A, var = 32, 100, 12, 0.3
        arms = np.random.RandomState(1234 + d).normal(size=(A, d)) / np.sqrt(d)
        thetas = np.random.RandomState(40 + d).normal(0, 1, (N, d)) / np.sqrt(d)
        envs = [bandit_env.LinearBanditEnv(t, arms, H, var=var) for t in thetas]
        vec = bandit_env.BanditEnvVec(envs)
        np.random.seed(50 + d)
        with DrawRecorder(np) as rec:
            cm, meta = eval_linear_bandit.deploy_online_vec(vec, cb.LinUCBPolicy(envs[0], const=1.0, batch_size=N),
                                                            H, include_meta=True)
        pre = f"d{d}/"
        out.update({pre + "means": np.stack([e.means for e in envs]), pre + "arms": arms, pre + "theta": thetas,
                    pre + "cum_means": cm, pre + "actions": meta["context_actions"].argmax(-1).astype(np.int8),
                    pre + "g": np.array(rec.g).reshape(H, N), pre + "first_action": np.asarray(rec.plain[0])})
    np.savez_compressed(os.path.join(OUT, "linucb_dims.npz"), **out)
    print("LinUCB dims")


def linear_offline():
    """evals/eval_linear_bandit.py:202-286 (offline: Opt, the DPT greedy leg, Thompson with the
    100-draw vote and prior 0/1, LinUCB with const 0 'linreg') on fixed contexts of 20-arm linear
    bandits, at every context length 1..Hc as offline_graph (:289-339) sweeps them.  The vote's
    posterior normals are recorded per call; returns are the dict offline() hands back."""
    import numpy as np
    import torch
    from envs import bandit_env
    from evals import eval_linear_bandit
    model = fixture_transformer("linear20")
    N, Hc, A, d, var = 10, 12, 20, 2, 0.3
    rs = np.random.RandomState(61)
    arms = np.random.RandomState(1234).normal(size=(A, d)) / np.sqrt(d)
    thetas = rs.normal(0, 1, (N, d)) / np.sqrt(d)
    trajs = []
    for t in thetas:
        env = bandit_env.LinearBanditEnv(t, arms, Hc, var=var)
        a = rs.randint(0, A, Hc)
        trajs.append({"theta": t, "arms": arms, "means": env.means, "context_states": np.ones((Hc, 1)),
                      "context_actions": np.eye(A)[a], "context_next_states": np.ones((Hc, 1)),
                      "context_rewards": env.means[a] + 0.3 * rs.normal(size=Hc)})
    out = {"theta": thetas, "arms": arms, "var": np.float64(var)}
    for k in ("context_actions", "context_rewards"):
        out[k] = np.stack([t[k] for t in trajs])
    for h in range(1, Hc + 1):
        np.random.seed(300 + h)
        with DrawRecorder(np) as rec, torch.no_grad():
            b = eval_linear_bandit.offline(trajs, model, n_eval=N, horizon=h, var=var)
        assert sorted(b) == ["linreg", "lnr", "opt", "thmp"] and len(rec.garr) == 100
        out[f"h{h}/vote_g"] = np.stack(rec.garr)  # (100, N, A)
        for k, v in b.items():
            out[f"h{h}/{k}"] = np.asarray(v)
    np.savez_compressed(os.path.join(OUT, "linear_offline.npz"), **out)
    print("linear offline")


def main():
    if not os.path.isdir(REF):
        raise SystemExit("reference checkout not present; fixtures are committed")
    _install_stubs()
    if len(sys.argv) > 1:  # regenerate only the named groups, e.g. `gen_golden.py baselines`
        import matplotlib
        matplotlib.use("Agg")
        sys.path[:0] = [REF, os.path.join(REF, "models")]
        for name in sys.argv[1:]:
            globals()[name]()
        return
    import matplotlib
    matplotlib.use("Agg")
    sys.path[:0] = [REF, os.path.join(REF, "models")]
    import numpy as np
    import torch
    torch.set_num_threads(8)
    from net import Transformer  # models/net.py:9
    from envs import bandit_env, darkroom_env
    from ctrls.ctrl_bandit import BanditTransformerController
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from evals import eval_bandit, eval_darkroom, eval_linear_bandit
    import collect_data

    # ---------------------------------------------------------------- F1 bandit transit
    rs = np.random.RandomState(11)
    N, A = 64, 5
    means = rs.uniform(0, 1, (N, A))
    act = rs.randint(0, A, N)
    out = {"means": means, "action": act}
    for var in (0.0, 0.3, 1.0):
        np.random.seed(100 + int(var * 10))
        with DrawRecorder(np) as rec:
            rew = []
            for i in range(N):
                env = bandit_env.BanditEnv(means[i], 1, var=var)
                u = np.zeros(A)
                u[act[i]] = 1.0
                env.reset()
                _, r, done, _ = env.step(u)  # envs/bandit_env.py:66-74
                assert done
                rew.append(r)
        out[f"g_var{var}"] = np.array(rec.g)
        out[f"reward_var{var}"] = np.array(rew, dtype=np.float64)
    # linear bandit: means = arms @ theta (envs/bandit_env.py:158-161)
    arms = np.random.RandomState(1234).normal(size=(20, 2)) / np.sqrt(2)
    thetas = rs.normal(0, 1, (16, 2)) / np.sqrt(2)
    lin_means = np.stack([bandit_env.LinearBanditEnv(t, arms, 10, var=0.3).means for t in thetas])
    out.update(lin_arms=arms, lin_theta=thetas, lin_means=lin_means,
               lin_opt=np.array([bandit_env.LinearBanditEnv(t, arms, 10).opt_a_index for t in thetas]))
    # arm value = np.sum(means * onehot) (envs/bandit_env.py:151-153)
    vec = bandit_env.BanditEnvVec([bandit_env.BanditEnv(m, 1) for m in means])
    onehot = np.eye(A)[act]
    out["arm_value"] = vec.get_arm_value(onehot)
    out["opt_index"] = np.array([e.opt_a_index for e in vec.envs])
    np.savez_compressed(os.path.join(OUT, "bandit_transit.npz"), **out)
    print("F1 bandit_transit")

    # ---------------------------------------------------------------- F2 darkroom table
    dim = 10
    states = np.array([(x, y) for x in range(dim) for y in range(dim)])
    nxt = np.zeros((100, 5, 100, 2), np.int8)
    rew = np.zeros((100, 5, 100), np.int8)
    opt = np.zeros((100, 100), np.int8)
    for gi, goal in enumerate(states):
        env = darkroom_env.DarkroomEnv(dim, goal, 100)
        for si, s in enumerate(states):
            opt[gi, si] = np.argmax(env.opt_action(s))
            for a in range(5):
                ns, r = env.transit(s, np.eye(5)[a])  # envs/darkroom_env.py:37-55
                nxt[gi, a, si] = ns
                rew[gi, a, si] = r
    pn = np.zeros((120, 5, 100, 2), np.int8)
    pr = np.zeros((120, 5, 100), np.int8)
    popt = np.zeros((120, 100), np.int8)
    perms = np.zeros((120, 5), np.int8)
    for pi in range(120):
        env = darkroom_env.DarkroomEnvPermuted(dim, pi, 100)
        perms[pi] = env.perm
        for si, s in enumerate(states):
            popt[pi, si] = np.argmax(env.opt_action(s))
            for a in range(5):
                ns, r = env.transit(s, np.eye(5)[a])
                pn[pi, a, si] = ns
                pr[pi, a, si] = r
    np.savez_compressed(os.path.join(OUT, "darkroom_transit.npz"), states=states,
                        next_state=nxt, reward=rew, opt_action=opt, perms=perms,
                        perm_next_state=pn, perm_reward=pr, perm_opt_action=popt)
    print("F2 darkroom_transit")

    # ---------------------------------------------------------------- F3 forward logits
    def make_model(sd_, ad, H, L=4, seed=0):
        cfg = dict(horizon=H, state_dim=sd_, action_dim=ad, n_layer=L, n_embd=32,
                   n_head=4, dropout=0.0, test=True)
        m = Transformer(cfg)
        w = perturbed_state_dict(m, seed)
        m.eval()
        return m, w, cfg

    def rand_context(rs, n, t, sd_, ad, kind):
        if kind == "darkroom":
            cs = rs.randint(0, 10, (n, t, sd_)).astype(np.float64)
            cn = rs.randint(0, 10, (n, t, sd_)).astype(np.float64)
            cr = (rs.uniform(size=(n, t, 1)) < 0.1).astype(np.float64)
            q = rs.randint(0, 10, (n, sd_)).astype(np.float64)
        else:
            cs = np.ones((n, t, sd_))
            cn = np.ones((n, t, sd_))
            cr = rs.normal(0.5, 0.5, (n, t, 1))
            q = np.ones((n, sd_))
        ca = np.eye(ad)[rs.randint(0, ad, (n, t))]
        return q, cs, ca, cn, cr

    models = {}
    for name, sd_, ad, H, Ts, kind in (
            ("bandit5", 1, 5, 500, (1, 2, 8, 101, 501), "bandit"),
            ("darkroom", 2, 5, 100, (1, 2, 8, 101), "darkroom"),
            ("linear20", 1, 20, 200, (1, 8, 201), "bandit")):
        model, w, cfg = make_model(sd_, ad, H, seed={"bandit5": 5, "darkroom": 10, "linear20": 20}[name])
        models[name] = (model, cfg)
        out = {f"w/{k}": v for k, v in w.items()}
        out["cfg"] = np.array([H, sd_, ad, 4, 32])
        rs = np.random.RandomState(7)
        for T in Ts:
            q, cs, ca, cn, cr = rand_context(rs, 16, T - 1, sd_, ad, kind)
            batch = {
                "query_states": torch.tensor(q).float(),
                "zeros": torch.zeros(16, sd_ ** 2 + ad + 1),
                "context_states": torch.tensor(cs).float(),
                "context_actions": torch.tensor(ca).float(),
                "context_next_states": torch.tensor(cn).float(),
                "context_rewards": torch.tensor(cr).float(),
            }
            with torch.no_grad():
                model.test = True
                logits = model(batch).numpy()
                model.test = False
                allp = model(batch).numpy()  # models/net.py:60 preds[:, 1:]
                model.test = True
            out.update({f"T{T}/query": q, f"T{T}/cs": cs, f"T{T}/ca": ca, f"T{T}/cn": cn,
                        f"T{T}/cr": cr, f"T{T}/logits": logits, f"T{T}/preds_train": allp})
        np.savez_compressed(os.path.join(OUT, f"forward_{name}.npz"), **out)
        print("F3 forward", name)

    # ---------------------------------------------------------------- F4 selection
    out = {}
    for A_, n in ((5, 512), (20, 256)):
        rs = np.random.RandomState(3 + A_)
        logits = (rs.normal(0, 2.0, (n, A_))).astype(np.float32)

        class _Stub(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.config = {"action_dim": A_, "state_dim": 1}
                self.horizon = 10

            def forward(self, batch):
                return torch.from_numpy(logits)

        ctrl = BanditTransformerController(_Stub(), sample=True, batch_size=n)
        ctrl.set_batch({})
        np.random.seed(2024 + A_)
        with DrawRecorder(np) as rec:
            oh = ctrl.act_numpy_vec([np.array([1])] * n)  # ctrls/ctrl_bandit.py:422-444
        out[f"A{A_}/logits"] = logits
        out[f"A{A_}/u"] = np.array(rec.u)
        out[f"A{A_}/sampled"] = oh.argmax(-1)
        ctrl.sample = False
        out[f"A{A_}/greedy"] = ctrl.act_numpy_vec([np.array([1])] * n).argmax(-1)
    np.savez_compressed(os.path.join(OUT, "select.npz"), **out)
    print("F4 select")

    # ---------------------------------------------------------------- F5 bandit rollouts
    def bandit_rollout(model, ad, n, H, var, sample, seed, linear=False):
        rs = np.random.RandomState(seed)
        if linear:
            arms = np.random.RandomState(1234).normal(size=(ad, 2)) / np.sqrt(2)
            thetas = rs.normal(0, 1, (n, 2)) / np.sqrt(2)
            envs = [bandit_env.LinearBanditEnv(t, arms, H, var=var) for t in thetas]
            mod = eval_linear_bandit
        else:
            means = rs.uniform(0, 1, (n, ad))
            envs = [bandit_env.BanditEnv(m, H, var=var) for m in means]
            mod = eval_bandit
        vec = bandit_env.BanditEnvVec(envs)
        ctrl = BanditTransformerController(model, sample=sample, batch_size=n)
        logs = []
        orig_fwd = model.forward

        def fwd(batch):
            o = orig_fwd(batch)
            logs.append(o.detach().numpy().copy())
            return o

        model.forward = fwd
        np.random.seed(seed + 1)
        try:
            with DrawRecorder(np) as rec, torch.no_grad():
                cm, meta = mod.deploy_online_vec(vec, ctrl, H, include_meta=True)
        finally:
            model.forward = orig_fwd
        res = {"means": np.stack([e.means for e in envs]), "cum_means": cm,
               "logits": np.stack(logs), "ctx_actions": meta["context_actions"],
               "ctx_rewards": meta["context_rewards"][..., 0],
               "ctx_states": meta["context_states"], "ctx_next_states": meta["context_next_states"],
               "cfg": np.array([n, H, ad, int(sample)]), "var": np.float64(var)}
        res["u"] = np.array(rec.u).reshape(H, n) if sample else np.zeros((H, n))
        res["g"] = np.array(rec.g).reshape(H, n)
        if linear:
            res["arms"] = arms
            res["theta"] = np.stack([e.theta for e in envs])
        return res

    m5, _ = models["bandit5"]
    for tag, kw in (("sample", dict(sample=True, var=0.3)), ("greedy", dict(sample=False, var=0.3)),
                    ("var0", dict(sample=True, var=0.0))):
        r = bandit_rollout(m5, 5, 8, 40, seed=31, **kw)
        np.savez_compressed(os.path.join(OUT, f"rollout_bandit_{tag}.npz"), **r)
    m20, _ = models["linear20"]
    r = bandit_rollout(m20, 20, 6, 24, 0.3, True, 41, linear=True)
    np.savez_compressed(os.path.join(OUT, "rollout_linear_sample.npz"), **r)
    print("F5 bandit rollouts")

    # online regret math on the Opt + Lnr legs (evals/eval_bandit.py:123-178)
    import scipy.stats
    r = dict(np.load(os.path.join(OUT, "rollout_bandit_sample.npz")))
    opt = np.stack([r["means"].max(-1)] * r["cum_means"].shape[0])  # Opt leg: means[opt_a]
    diff = (opt - r["cum_means"]).T
    cr = np.cumsum(diff, axis=1)
    np.savez_compressed(os.path.join(OUT, "regret_math.npz"), lnr=r["cum_means"].T, opt=opt.T,
                        subopt_mean=np.mean(diff, 0), subopt_sem=scipy.stats.sem(diff, 0),
                        regret_mean=np.mean(cr, 0), regret_sem=scipy.stats.sem(cr, 0))

    # ---------------------------------------------------------------- offline greedy (var=0 deploy_eval)
    rs = np.random.RandomState(51)
    n, h = 8, 50
    means = rs.uniform(0, 1, (n, 5))
    envs = [bandit_env.BanditEnv(m, h, var=0.3) for m in means]
    vec = bandit_env.BanditEnvVec(envs)
    ca = np.eye(5)[rs.randint(0, 5, (n, h))]
    cr = (means[np.arange(n)[:, None], ca.argmax(-1)] + 0.3 * rs.normal(size=(n, h)))[..., None]
    batch = {"context_states": np.ones((n, h, 1)), "context_actions": ca,
             "context_next_states": np.ones((n, h, 1)), "context_rewards": cr}
    ctrl = BanditTransformerController(m5, sample=False, batch_size=n)
    ctrl.set_batch_numpy_vec(batch)
    with torch.no_grad():
        _, us, _, rs_ = vec.deploy_eval(ctrl)  # envs/bandit_env.py:114-123 (var forced to 0)
    np.savez_compressed(os.path.join(OUT, "offline_bandit.npz"), means=means, ctx_actions=ca,
                        ctx_rewards=cr[..., 0], actions=us.argmax(-1), rewards=rs_)
    print("F5b offline")

    # ---------------------------------------------------------------- F6 darkroom rollouts
    mdr, _ = models["darkroom"]

    def darkroom_rollout(n, Heps, H, horizon, sample, seed, permuted=False):
        rs = np.random.RandomState(seed)
        if permuted:
            idx = rs.randint(0, 120, n)
            envs = [darkroom_env.DarkroomEnvPermuted(10, int(i), horizon) for i in idx]
        else:
            goals = rs.randint(0, 10, (n, 2))
            envs = [darkroom_env.DarkroomEnv(10, g, horizon) for g in goals]
        vec = darkroom_env.DarkroomEnvVec(envs)
        ctrl = DarkroomTransformerController(mdr, batch_size=n, sample=sample)
        logs = []
        orig_fwd = mdr.forward

        def fwd(batch):
            o = orig_fwd(batch)
            logs.append(o.detach().numpy().copy())
            return o

        mdr.forward = fwd
        np.random.seed(seed + 1)
        try:
            with DrawRecorder(np) as rec, torch.no_grad():
                ret = eval_darkroom.deploy_online_vec(vec, ctrl, Heps, H, horizon)
        finally:
            mdr.forward = orig_fwd
        res = {"goals": np.stack([e.goal for e in envs]), "returns": ret,
               "logits": np.stack(logs), "cfg": np.array([n, Heps, H, horizon, int(sample)])}
        res["u"] = (np.array(rec.u).reshape(Heps, horizon, n) if sample
                    else np.zeros((Heps, horizon, n)))
        if permuted:
            res["perm_index"] = idx
        return res

    for tag, kw in (("sample", dict(sample=True)), ("greedy", dict(sample=False))):
        r = darkroom_rollout(6, 5, 20, 10, seed=61, **kw)
        np.savez_compressed(os.path.join(OUT, f"rollout_darkroom_{tag}.npz"), **r)
    r = darkroom_rollout(4, 3, 10, 10, True, 71, permuted=True)
    np.savez_compressed(os.path.join(OUT, "rollout_darkroom_permuted.npz"), **r)
    print("F6 darkroom rollouts")

    # ---------------------------------------------------------------- F7 rollin (collect_data)
    np.random.seed(0)
    out = {}
    for i in range(6):
        env = bandit_env.sample(5, 20, 0.3)  # envs/bandit_env.py:10-18
        rec_vals = {}
        real_dir = np.random.dirichlet

        def dirichlet(alpha, _r=real_dir):
            v = _r(alpha)
            rec_vals["probs"] = v
            return v

        np.random.dirichlet = dirichlet
        try:
            with DrawRecorder(np) as rec:
                xs, us, xps, rs_ = collect_data.rollin_bandit(env, cov=0.0)
            # the two no-p choices: cov pick, then the random arm (collect_data.py:30-35)
            picks = rec.plain
        finally:
            np.random.dirichlet = real_dir
        out[f"{i}/means"] = env.means
        out[f"{i}/cov"] = np.float64(picks[0])
        out[f"{i}/dirichlet"] = rec_vals["probs"]
        out[f"{i}/rand_index"] = np.int64(picks[1])
        out[f"{i}/u"] = np.array(rec.u)
        out[f"{i}/g"] = np.array(rec.g)
        out[f"{i}/xs"], out[f"{i}/us"], out[f"{i}/xps"], out[f"{i}/rs"] = xs, us, xps, rs_
    # rollin_mdp (uniform): draws are the sampled (state, action) pairs themselves
    np.random.seed(1)
    env = darkroom_env.DarkroomEnv(10, np.array([3, 7]), 12)
    s, a, ns, r = collect_data.rollin_mdp(env, "uniform")  # collect_data.py:83-111
    out.update({"mdp/states": s, "mdp/actions": a, "mdp/next_states": ns, "mdp/rewards": r,
                "mdp/goal": env.goal})
    np.savez_compressed(os.path.join(OUT, "rollin.npz"), **out)
    print("F7 rollin")


if __name__ == "__main__":
    main()
