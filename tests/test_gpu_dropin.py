"""The reference-named drop-in layer (envs/, ctrls/, evals/, models/, collect_data) on the GPU,
against golden vectors recorded from the reference and the oracle."""
import os

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import dpt_oracle as O

pytestmark = pytest.mark.gpu


def ref_model(name, horizon=None):
    """models.net.Transformer loaded (strict) from a reference state_dict fixture; a shorter
    ``horizon`` keeps the first 4(1+horizon) wpe rows (gen_golden.fixture_transformer)."""
    from models.net import Transformer
    g = golden(f"forward_{name}.npz")
    H, sd, A, L, E = (int(x) for x in g["cfg"])
    horizon = horizon or H
    m = Transformer(dict(horizon=horizon, state_dim=sd, action_dim=A, n_layer=L, n_embd=E, n_head=4, dropout=0.0,
                         test=True))
    state = {k[2:]: torch.from_numpy(v[: 4 * (1 + horizon)] if k.endswith("wpe.weight") else v)
             for k, v in g.items() if k.startswith("w/")}
    state["transformer.wte.weight"] = m.transformer.wte.weight.detach().clone()
    state["transformer.h.0.attn.bias"] = torch.ones(1)  # transformers 4.5.1 legacy buffer: dropped on load
    m.load_state_dict(state)
    m.eval()  # as eval.py:152 does
    return g, m


def test_transformer_forward_drop_in():
    g, m = ref_model("darkroom")
    for T in (1, 8, 101):
        b = {"query_states": torch.from_numpy(g[f"T{T}/query"]).float(),
             "zeros": torch.zeros(16, 2 ** 2 + 5 + 1)}
        if T > 1:
            b.update(context_states=torch.from_numpy(g[f"T{T}/cs"]).float(),
                     context_actions=torch.from_numpy(g[f"T{T}/ca"]).float(),
                     context_next_states=torch.from_numpy(g[f"T{T}/cn"]).float(),
                     context_rewards=torch.from_numpy(g[f"T{T}/cr"]).float())
        else:
            b.update(context_states=torch.zeros(16, 0, 2), context_actions=torch.zeros(16, 0, 5),
                     context_next_states=torch.zeros(16, 0, 2), context_rewards=torch.zeros(16, 0, 1))
        out = m(b).cpu().numpy()
        ref = g[f"T{T}/logits"]
        assert (np.abs(out - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all()
    # parameter change -> device weights repacked
    with torch.no_grad():
        m.pred_actions.bias += 1.0
    out2 = m(b).cpu().numpy()
    assert np.allclose(out2, out + 1.0, atol=1e-5)


@pytest.mark.parametrize("tag", ["sample", "greedy"])
def test_eval_bandit_deploy_online_vec(tag):
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    r = golden(f"rollout_bandit_{tag}.npz")
    _, m = ref_model("bandit5")
    n, H, A, sample = (int(x) for x in r["cfg"])
    envs = [BanditEnv(mu, H, var=float(r["var"])) for mu in r["means"]]
    vec = BanditEnvVec(envs)
    ctrl = BanditTransformerController(m, sample=bool(sample), batch_size=n)
    cm, meta = eval_bandit.deploy_online_vec(vec, ctrl, H, include_meta=True, uniforms=r["u"] if sample else None,
                                             noise=r["g"])
    assert np.array_equal(cm, r["cum_means"])
    for k, ref in (("context_actions", r["ctx_actions"]), ("context_states", r["ctx_states"]),
                   ("context_next_states", r["ctx_next_states"])):
        assert np.array_equal(meta[k], ref), k
    assert np.array_equal(meta["context_rewards"][..., 0], r["ctx_rewards"])


def test_generic_loop_equals_fused():
    """The reference per-step loop (controller stepped through envs on device) and the fused
    kernel give the same trajectory for the same injected draws."""
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    r = golden("rollout_bandit_greedy.npz")
    _, m = ref_model("bandit5")
    n, H = 8, 12
    envs = [BanditEnv(mu, H, var=0.0) for mu in r["means"]]
    vec = BanditEnvVec(envs)

    cm_f = eval_bandit.deploy_online_vec(vec, BanditTransformerController(m, sample=False, batch_size=n), H)
    cm_g = eval_bandit.deploy_online_vec(vec, BanditTransformerController(m, sample=False, batch_size=n), H,
                                         fused=False)
    assert np.array_equal(cm_f, cm_g)
    # classical policies: per-step prefix-context kernel calls == fused kernel (var=0: no env noise);
    # Thompson's posterior draws come from the controller's stream in both loops (Philox counter
    # k of one seed at step k), or from the injected policy_noise
    from ctrls.ctrl_bandit import EmpMeanPolicy, PessMeanPolicy, ThompsonSamplingPolicy, UCBPolicy

    def thompson(sample, counter=0, pn=None):
        c = ThompsonSamplingPolicy(envs[0], std=0.3, sample=sample, prior_mean=0.5, prior_var=1 / 12.0,
                                   batch_size=n)
        c._stream.seed, c._stream.counter = 777, counter
        c.policy_noise = pn
        return c

    pg = np.random.RandomState(4).standard_normal((40, n, 5))
    for mk in (lambda: EmpMeanPolicy(envs[0], online=True, batch_size=n), lambda: UCBPolicy(envs[0], batch_size=n),
               lambda: PessMeanPolicy(envs[0], const=0.8, batch_size=n), lambda: thompson(True),
               lambda: thompson(True, 9), lambda: thompson(False, 3), lambda: thompson(True, 2, lambda k: pg[k])):
        ca, cb = mk(), mk()
        a = eval_bandit.deploy_online_vec(vec, ca, H)
        b = eval_bandit.deploy_online_vec(vec, cb, H, fused=False)
        assert np.array_equal(a, b), type(ca).__name__
        assert ca._stream.counter == cb._stream.counter
    # injected posterior normals are the ones used: equal to the kernel fed them directly
    import dpt_hip
    out = dpt_hip.rollout_policy(dpt_hip.POLICY_THOMPSON, r["means"], H, 0.0, ts_std=0.3, ts_prior_mean=0.5,
                                 ts_prior_var=1 / 12.0, policy_noise=pg[2:2 + H])
    assert np.array_equal(out["arm_value"].cpu().numpy().T,
                          eval_bandit.deploy_online_vec(vec, thompson(True, 2, lambda k: pg[k]), H))


def test_fused_bandit_uses_controller_stream():
    """The fused bandit rollout draws its selection uniforms from the controller's own stream:
    fused and per-step loops act on the same Philox draws (var=0: no env noise), the stream
    advances by H either way, and uniforms injected on the controller are used by both."""
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    _, m = ref_model("bandit5")
    rs = np.random.RandomState(12)
    n, H = 24, 16
    envs = [BanditEnv(rs.uniform(0, 1, 5), H, var=0.0) for _ in range(n)]
    vec = BanditEnvVec(envs)

    def ctrl(counter=0, uniforms=None):
        c = BanditTransformerController(m, sample=True, batch_size=n)
        c._stream.seed, c._stream.counter = 4242, counter
        c.uniforms = uniforms
        return c

    for counter in (0, 37):
        cf, cg = ctrl(counter), ctrl(counter)
        a_f = eval_bandit.deploy_online_vec(vec, cf, H, include_meta=True)[1]["context_actions"]
        a_g = eval_bandit.deploy_online_vec(vec, cg, H, include_meta=True, fused=False)[1]["context_actions"]
        assert np.array_equal(a_f, a_g), counter
        assert cf._stream.counter == cg._stream.counter == counter + H
    u = rs.uniform(size=(100, n))
    cf, cg = ctrl(5, lambda k: u[k]), ctrl(5, lambda k: u[k])
    a_f = eval_bandit.deploy_online_vec(vec, cf, H, include_meta=True)[1]["context_actions"]
    a_g = eval_bandit.deploy_online_vec(vec, cg, H, include_meta=True, fused=False)[1]["context_actions"]
    assert np.array_equal(a_f, a_g)
    # explicit uniforms override the controller's; counters 5..5+H of u are the ones used
    out = eval_bandit.rollout_fused(vec, ctrl(0), H, uniforms=u[5:5 + H])
    assert np.array_equal(np.eye(5)[out["actions"].cpu().numpy()], a_f)


def test_offline_greedy_matches_reference():
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    r = golden("offline_bandit.npz")
    _, m = ref_model("bandit5")
    n, h = r["ctx_actions"].shape[:2]
    envs = [BanditEnv(mu, h, var=0.3) for mu in r["means"]]
    vec = BanditEnvVec(envs)
    ctrl = BanditTransformerController(m, sample=False, batch_size=n)
    ctrl.set_batch_numpy_vec({"context_states": np.ones((n, h, 1)), "context_actions": r["ctx_actions"],
                              "context_next_states": np.ones((n, h, 1)), "context_rewards": r["ctx_rewards"][..., None]})
    _, us, _, rs = vec.deploy_eval(ctrl)
    assert np.array_equal(us.argmax(-1), r["actions"])
    assert np.array_equal(rs, r["rewards"])  # var forced to 0: rewards = means[a] exactly


@pytest.mark.parametrize("name", ["emp", "ucb", "thomp"])
def test_baseline_policy_kernel(name):
    import dpt_hip
    g = golden("baselines.npz")
    code = {"emp": dpt_hip.POLICY_EMP, "ucb": dpt_hip.POLICY_UCB, "thomp": dpt_hip.POLICY_THOMPSON}[name]
    kw = dict(online=True, c=1.0, ts_std=0.3, ts_prior_mean=0.5, ts_prior_var=1 / 12.0)
    H = g[f"{name}/g"].shape[0]
    out = dpt_hip.rollout_policy(code, g["means"], H, 0.3, noise=g[f"{name}/g"],
                                 policy_noise=g.get(f"{name}/policy_g"), **kw)
    assert np.array_equal(out["actions"].cpu().numpy(), g[f"{name}/actions"])
    assert np.array_equal(out["rewards"].cpu().numpy(), g[f"{name}/rewards"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, g[f"{name}/cum_means"])


def test_baseline_offline_prefix_and_linucb():
    import dpt_hip
    g = golden("baselines.npz")
    ca, cr = g["off/ctx_actions"], g["off/ctx_rewards"]
    for name, code, c in (("emp", dpt_hip.POLICY_EMP, 1.0), ("lcb", dpt_hip.POLICY_LCB, 0.8)):
        out = dpt_hip.rollout_policy(code, g["means"], 1, 0.0, online=False, c=c, ctx_actions=ca, ctx_rewards=cr)
        assert np.array_equal(out["actions"][:, 0].cpu().numpy(), g[f"off/{name}/actions"])
    A = g["lin/arms"].shape[0]
    u = (g["lin/first_action"] + 0.5) / A
    H = g["lin/g"].shape[0]
    out = dpt_hip.rollout_policy(dpt_hip.POLICY_LINUCB, g["lin/means"], H, 0.3, c=1.0, arms=g["lin/arms"],
                                 noise=g["lin/g"], policy_noise=u)
    acts = out["actions"].cpu().numpy()
    # LinUCB restates numpy's BLAS/LAPACK rounding order (dpt_policies.hip linucb_choose): exact
    assert np.array_equal(acts, g["lin/actions"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, g["lin/cum_means"])


@pytest.mark.parametrize("fix", ["linucb_d4", "linucb_long", "linucb_dims:3", "linucb_dims:5", "linucb_dims:6",
                                 "linucb_dims:8"])
def test_linucb_kernel_and_drop_in(fix):
    """LinUCB (ctrls/ctrl_bandit.py:447-528) against the reference's recorded online runs: lin_d = 4
    (12 arms, 20 steps), lin_d = 2 on the C4 arm table over 800 steps (the context crosses the
    BLAS blocking of X^T X at 384 and 768 rows), and lin_d 3 / 5 / 6 / 8 over 100 steps (the
    numpy orders of dpt_linucb.h at every width the kernel takes).  Every arm index and arm value
    exactly, through the kernel and through eval_linear_bandit.deploy_online_vec with the
    reference's draws injected."""
    import dpt_hip
    from ctrls.ctrl_bandit import LinUCBPolicy
    from envs.bandit_env import BanditEnvVec, LinearBanditEnv
    from evals import eval_linear_bandit
    if ":" in fix:
        name, d = fix.split(":")
        gz = golden(f"{name}.npz")
        g = {k.split("/", 1)[1]: gz[k] for k in gz if k.startswith(f"d{d}/")}
    else:
        g = golden(f"{fix}.npz")
    A = g["arms"].shape[0]
    H = g["g"].shape[0]
    u = (g["first_action"] + 0.5) / A
    out = dpt_hip.rollout_policy(dpt_hip.POLICY_LINUCB, g["means"], H, 0.3, c=1.0, arms=g["arms"], noise=g["g"],
                                 policy_noise=u)
    acts = out["actions"].cpu().numpy()
    assert np.array_equal(acts, g["actions"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, g["cum_means"])
    envs = [LinearBanditEnv(t, g["arms"], H, var=0.3) for t in g["theta"]]
    assert np.array_equal(np.stack([e.means for e in envs]), g["means"])
    vec = BanditEnvVec(envs)
    ctrl = LinUCBPolicy(envs[0], const=1.0, batch_size=len(envs))
    pn = np.zeros((H, len(envs)))
    pn[0] = u
    cm, meta = eval_linear_bandit.deploy_online_vec(vec, ctrl, H, include_meta=True, noise=g["g"], policy_noise=pn)
    assert np.array_equal(meta["context_actions"].argmax(-1), g["actions"])
    assert np.array_equal(cm, g["cum_means"])


def test_linear_offline_and_graph_match_reference():
    """evals/eval_linear_bandit.py offline (:202-286) and offline_graph (:289-339) against the
    reference's recorded results at every context length 1..12: the opt / lnr (DPT greedy) /
    thmp (100-draw vote, prior 0 / 1, the reference's posterior normals injected) / linreg
    (LinUCB, const 0) rewards exactly, and offline_graph's sweep over np.linspace(1, H, H)."""
    import matplotlib
    matplotlib.use("Agg")
    from evals import eval_linear_bandit as elb
    g = golden("linear_offline.npz")
    _, m = ref_model("linear20")
    N, Hc = g["context_rewards"].shape
    trajs = [{"theta": g["theta"][i], "arms": g["arms"], "context_states": np.ones((Hc, 1)),
              "context_actions": g["context_actions"][i], "context_next_states": np.ones((Hc, 1)),
              "context_rewards": g["context_rewards"][i]} for i in range(N)]
    calls = []

    class TS(elb.ThompsonSamplingPolicy):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            h = len(calls) % Hc + 1  # offline() builds one Thompson controller per context length
            calls.append(h)
            self.policy_noise = lambda ctr: g[f"h{h}/vote_g"]

    orig = elb.ThompsonSamplingPolicy
    elb.ThompsonSamplingPolicy = TS
    try:
        for h in range(1, Hc + 1):
            b = elb.offline(trajs, m, n_eval=N, horizon=h, var=float(g["var"]))
            assert list(b) == ["opt", "lnr", "thmp", "linreg"]
            for k, v in b.items():
                assert np.array_equal(v, g[f"h{h}/{k}"]), (h, k)
        horizons, allb = elb.offline_graph(trajs, m, n_eval=N, horizon=Hc, var=float(g["var"]))
    finally:
        elb.ThompsonSamplingPolicy = orig
    assert np.array_equal(horizons, np.arange(1, Hc + 1))
    for h, b in zip(horizons, allb):
        for k, v in b.items():
            assert np.array_equal(v, g[f"h{h}/{k}"]), (h, k)


def test_online_and_offline_eval_run():
    import matplotlib
    matplotlib.use("Agg")
    from evals import eval_bandit
    _, m = ref_model("bandit5")
    rs = np.random.RandomState(3)
    trajs = [{"means": rs.uniform(0, 1, 5), "context_states": np.ones((30, 1)),
              "context_actions": np.eye(5)[rs.randint(0, 5, 30)], "context_next_states": np.ones((30, 1)),
              "context_rewards": rs.normal(0.5, 0.3, 30)} for _ in range(16)]
    np.random.seed(0)
    all_means, st = eval_bandit.online(trajs, m, n_eval=16, horizon=30, var=0.3, bandit_type="uniform")
    assert set(all_means) == {"opt", "Lnr", "Emp", "UCB1.0", "Thomp"}
    assert all(v.shape == (16, 30) for v in all_means.values())
    assert (st["regret_means"]["opt"] == 0).all()
    base = eval_bandit.offline(trajs, m, n_eval=16, horizon=30, var=0.3, bandit_type="uniform")
    assert set(base) == {"opt", "lnr", "emp", "thmp", "lcb"}
    assert (base["opt"] >= base["lnr"] - 1e-12).all()


@pytest.mark.parametrize("fused", [True, False])
def test_eval_darkroom_device_loop_matches_reference(fused):
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvPermuted, DarkroomEnvVec
    from evals import eval_darkroom
    _, m = ref_model("darkroom")
    for tag in ("sample", "greedy", "permuted"):
        r = golden(f"rollout_darkroom_{tag}.npz")
        n, Heps, H, horizon, sample = (int(x) for x in r["cfg"])
        if tag == "permuted":
            envs = [DarkroomEnvPermuted(10, int(i), horizon) for i in r["perm_index"]]
        else:
            envs = [DarkroomEnv(10, g_, horizon) for g_ in r["goals"]]
        ctrl = DarkroomTransformerController(m, batch_size=n, sample=bool(sample))
        u = r["u"].reshape(-1, n)
        ctrl.uniforms = lambda k: u[k]
        vec = DarkroomEnvVec(envs)
        assert eval_darkroom._fused_ok(vec, ctrl, H) or not fused
        ret = eval_darkroom.deploy_online_vec(vec, ctrl, Heps, H, horizon, fused=fused)
        assert np.array_equal(ret, r["returns"]), tag


def test_eval_darkroom_per_step_memo_bit_identical():
    """The per-step device loop (fused=False, window 1 + 2*130 = 261) forwards only the tasks
    whose state is new in the episode; returns are identical with the memo off."""
    import dpt_hip
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec
    from evals import eval_darkroom
    _, m = ref_model("darkroom")
    rs = np.random.RandomState(8)
    envs = [DarkroomEnv(10, rs.randint(0, 10, 2), 130) for _ in range(48)]
    outs = []
    try:
        for memo in (False, True):
            dpt_hip.set_darkroom_memo(memo)
            np.random.seed(5)
            ctrl = DarkroomTransformerController(m, batch_size=48, sample=True)
            vec = DarkroomEnvVec(envs)
            outs.append(eval_darkroom.deploy_online_vec(vec, ctrl, 3, 260, 130, fused=False))
    finally:
        dpt_hip.set_darkroom_memo(True)
    assert np.array_equal(outs[0], outs[1])


def test_eval_darkroom_per_step_shard_invariant():
    """The per-step device loop (fused=False, window 1 + 2*130 = 261) keys its
    selection draws by the GLOBAL task id (DarkroomEnvVec.first_task), like the fused kernel:
    two shards of the tasks, each with the same controller seed, give the unsharded returns."""
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec
    from evals import eval_darkroom
    _, m = ref_model("darkroom")
    rs = np.random.RandomState(9)
    goals = [rs.randint(0, 10, 2) for _ in range(40)]

    def run(lo, hi):
        envs = [DarkroomEnv(10, g_, 130) for g_ in goals[lo:hi]]
        ctrl = DarkroomTransformerController(m, batch_size=hi - lo, sample=True)
        ctrl._stream.seed = 31337
        vec = DarkroomEnvVec(envs, first_task=lo)
        return eval_darkroom.deploy_online_vec(vec, ctrl, 3, 260, 130, fused=False)

    full = run(0, 40)
    assert np.array_equal(np.concatenate([run(0, 17), run(17, 40)]), full)


def test_rollin_kernels_match_oracle():
    import dpt_hip
    g = golden("rollin.npz")
    for i in range(6):
        means, cov, dr = g[f"{i}/means"], float(g[f"{i}/cov"]), g[f"{i}/dirichlet"]
        p = (1 - cov) * dr + cov * np.eye(5)[int(g[f"{i}/rand_index"])]
        u, gg = g[f"{i}/u"], g[f"{i}/g"]
        acts, rews = dpt_hip.rollin_bandit(means[None], p[None], len(u), 0.3, uniforms=u[:, None], noise=gg[:, None])
        assert np.array_equal(np.eye(5)[acts.cpu().numpy()[0]], g[f"{i}/us"])
        assert np.array_equal(rews.cpu().numpy()[0], g[f"{i}/rs"])
    s, a = g["mdp/states"], g["mdp/actions"].argmax(-1)
    o = dpt_hip.rollin_darkroom(g["mdp/goal"][None], len(a), 10, states=s[None], actions=a[None])
    assert np.array_equal(o["next_states"].cpu().numpy()[0], g["mdp/next_states"])
    assert np.array_equal(o["rewards"].cpu().numpy()[0], g["mdp/rewards"])
    # expert rollin walks to the goal: reward 1 from arrival on
    goals = np.array([[3, 7], [9, 9], [0, 0]])
    o = dpt_hip.rollin_darkroom(goals, 25, 10, mode=1)
    rw = o["rewards"].cpu().numpy()
    assert (rw[:, -1] == 1).all() and (rw[2] == 1).all()


def test_collect_data_generators_format():
    import collect_data
    from envs import bandit_env
    np.random.seed(0)
    trajs = collect_data.generate_bandit_histories(64, 5, 20, 0.3, n_hists=2, n_samples=2, cov=0.0, type="uniform")
    assert len(trajs) == 64 * 4
    t = trajs[0]
    assert set(t) == {"query_state", "optimal_action", "context_states", "context_actions", "context_next_states",
                      "context_rewards", "means"}
    assert t["context_actions"].shape == (20, 5) and t["context_actions"].dtype == np.float64
    assert t["context_states"].shape == (20, 1) and t["context_rewards"].shape == (20,)
    a = t["context_actions"].argmax(-1)
    noise = t["context_rewards"] - t["means"][a]
    assert np.abs(noise).max() < 0.3 * 6
    goals = np.array([[1, 2], [3, 4], [9, 9]])
    dtr = collect_data.generate_darkroom_histories(goals, 10, 30, n_hists=1, n_samples=3, rollin_type="uniform")
    assert len(dtr) == 9
    for t in dtr:
        ns, r = O.darkroom_transit(t["context_states"], t["context_actions"].argmax(-1),
                                   np.broadcast_to(t["goal"], (30, 2)))
        assert np.array_equal(ns, t["context_next_states"]) and np.array_equal(r, t["context_rewards"])
        q = t["query_state"][None]
        assert t["optimal_action"].argmax() == O.darkroom_opt_action(q, t["goal"][None])[0]
    lin = collect_data.generate_linear_bandit_histories(8, 10, 2, 12, 0.3, n_hists=1, n_samples=1, cov=0.0,
                                                        data_type="thompson")
    assert len(lin) == 8 and lin[0]["context_actions"].shape == (12, 10)
    assert isinstance(bandit_env.LinearBanditEnv(lin[0]["theta"], lin[0]["arms"], 12).means, np.ndarray)


def test_gpu_bandit_env():
    from envs.gpu_bandit_env import GPUBanditEnv
    torch.manual_seed(0)
    env = GPUBanditEnv(5, 64, 3, var=0.3)
    env.reset()
    us = torch.nn.functional.one_hot(torch.randint(0, 5, (64,)), 5).float().cuda()
    _, r, done, _ = env.step(us)
    assert r.dtype == torch.float32 and r.shape == (64,) and not bool(done.any())
    env.step(us)
    _, _, done, _ = env.step(us)
    assert bool(done.all())
    with pytest.raises(ValueError):
        env.step(us)
    m = env.means[torch.arange(64), us.argmax(1)]
    assert float((r - m).abs().max()) < 0.3 * 6


def test_cli_collect_then_eval(tmp_path, monkeypatch):
    """The reference command lines end to end (run_bandit.sh / run_darkroom.sh shape, small sizes):
    collect_data.py writes its dataset pickles under datasets/, a checkpoint of a fresh
    Transformer loads strictly, and eval.py runs online/offline evaluation and writes its figures."""
    import glob
    import importlib

    import matplotlib
    matplotlib.use("Agg")
    import collect_data
    from models.net import Transformer
    ev = importlib.import_module("eval")
    monkeypatch.chdir(tmp_path)
    runs = [
        ("bandit", 1, 5, ["--envs", "50", "--envs_eval", "8", "--H", "20", "--dim", "5", "--var", "0.3"],
         ["--n_eval", "8"]),
        ("linear_bandit", 1, 5, ["--envs", "50", "--envs_eval", "8", "--H", "20", "--dim", "5", "--lin_d", "2",
                                 "--var", "0.3"], ["--n_eval", "8"]),
        ("darkroom_heldout", 2, 5, ["--envs", "100", "--H", "20", "--dim", "10"], ["--n_eval", "100"]),
    ]
    for env, sd, A, data_args, eval_args in runs:
        collect_data.main(["--env", env] + data_args)
        assert len(glob.glob(f"datasets/*{env}*")) == 3, env
        H = int(data_args[data_args.index("--H") + 1])
        torch.manual_seed(0)
        model = Transformer(dict(horizon=H, state_dim=sd, action_dim=A, n_layer=3, n_embd=32, n_head=1,
                                 dropout=0.0, test=True))
        ckpt = tmp_path / f"{env}.pt"
        torch.save(model.state_dict(), ckpt)
        ev.main(["--env", env, "--checkpoint", str(ckpt)] + data_args + eval_args)
        figs = glob.glob("figs/evals_epoch-1/*/*.png")
        assert len(figs) >= 2, (env, figs)
        for f in figs:
            os.remove(f)


def test_c1_collect_and_eval_bit_exact():
    """BASELINE config 1 at its size (run_bandit.sh flags: 5 arms, var 0.3; 64 tasks, H=100):
    (a) the collect rollins of all 64 tasks in one dpt_rollin_bandit launch reproduce the
    reference's generate_bandit_histories draw for draw; (b) eval_bandit.deploy_online_vec with
    the DPT sampling controller reproduces the reference's cum_means, actions and rewards bit for
    bit, and the regret curves (evals/eval_bandit.py:169-178) from the device moments equal the
    reference's within 1e-12."""
    import dpt_hip
    from ctrls.ctrl_bandit import BanditTransformerController
    from dpt_hip.distributed import regret_stats_allreduce
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    g = golden("c1_bandit.npz")
    N, H, A = (int(x) for x in g["cfg"])
    cov = g["collect/cov"][:, None]
    p = (1 - cov) * g["collect/dirichlet"] + cov * np.eye(A)[g["collect/rand_index"]]
    acts, rews = dpt_hip.rollin_bandit(g["collect/means"], p, H, 0.3, uniforms=g["collect/u"].T,
                                       noise=g["collect/g"].T)
    assert np.array_equal(acts.cpu().numpy(), g["collect/actions"])
    assert np.array_equal(rews.cpu().numpy(), g["collect/rewards"])
    _, m = ref_model("bandit5", horizon=H)
    envs = [BanditEnv(mu, H, var=float(g["var"])) for mu in g["eval/means"]]
    vec = BanditEnvVec(envs)
    for fused in (True, False):
        ctrl = BanditTransformerController(m, sample=True, batch_size=N)
        cm, meta = eval_bandit.deploy_online_vec(vec, ctrl, H, include_meta=True, uniforms=g["eval/u"],
                                                 noise=g["eval/g"], fused=fused)
        assert np.array_equal(cm, g["eval/cum_means"]), fused
        assert np.array_equal(meta["context_actions"].argmax(-1), g["eval/actions"]), fused
        assert np.array_equal(meta["context_rewards"][..., 0], g["eval/rewards"]), fused
    opt = torch.from_numpy(g["eval/means"].max(1)).cuda()
    st = regret_stats_allreduce(opt, torch.from_numpy(cm.T.copy()).cuda(), N)
    for k in ("subopt_mean", "subopt_sem", "regret_mean", "regret_sem"):
        np.testing.assert_allclose(st[k].cpu().numpy(), g[f"eval/{k}"], rtol=1e-12, atol=1e-15)


def test_gpu_bandit_env_fp32_bit_exact():
    """GPUBanditEnv (envs/gpu_bandit_env.py:53-74) with the reference's torch.randn draws
    injected: fp32 rewards mean + g * var bit for bit, done flags, ValueError past H."""
    from envs.gpu_bandit_env import GPUBanditEnv
    g = golden("gpu_bandit_env.npz")
    for var in (0.3, 1.0):
        env = GPUBanditEnv(5, 64, 3, var=var)
        env.means = torch.from_numpy(g[f"var{var}/means"]).cuda()
        draws = g[f"var{var}/g"]
        env.noise = lambda k: draws[k]
        env.reset()
        for t in range(3):
            us = torch.nn.functional.one_hot(torch.from_numpy(g[f"var{var}/actions"][t]).long(), 5).float().cuda()
            _, r, done, _ = env.step(us)
            assert r.dtype == torch.float32
            assert np.array_equal(r.cpu().numpy().view(np.int32), g[f"var{var}/rewards"][t].view(np.int32)), (var, t)
            assert np.array_equal(done.cpu().numpy(), g[f"var{var}/done"][t])
        with pytest.raises(ValueError, match=str(g[f"var{var}/error"])):
            env.step(us)


def test_linear_thompson_rollin_bit_exact():
    """collect_data.rollin_linear_bandit_vec (collect_data.py:56-80: Thompson, prior N(0, 1), 10-arm
    linear bandits, lin_d = 2) with the reference's posterior and reward normals injected."""
    import collect_data
    from envs.bandit_env import LinearBanditEnv
    g = golden("linear_thompson.npz")
    H = g["g"].shape[0]
    envs = [LinearBanditEnv(t, g["arms"], H, var=float(g["var"])) for t in g["theta"]]
    assert np.array_equal(np.stack([e.means for e in envs]), g["means"])
    cs, ca, cn, cr = collect_data.rollin_linear_bandit_vec(envs, noise=g["g"], policy_noise=g["policy_g"])
    for got, k in ((cs, "context_states"), (ca, "context_actions"), (cn, "context_next_states"),
                   (cr, "context_rewards")):
        assert np.array_equal(got, g[k]), k


@pytest.mark.parametrize("tag", ["plain", "permuted"])
def test_darkroom_offline_matches_reference(tag):
    """eval_darkroom.offline (evals/eval_darkroom.py:124-189) on the reference's fixed contexts:
    the expert's returns, the greedy leg and the sampled leg (its uniforms injected) equal the
    reference's returns; per-step rewards through the same device episode."""
    import matplotlib
    matplotlib.use("Agg")
    import dpt_hip
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvPermuted, DarkroomEnvVec
    from evals import eval_darkroom
    g = golden("darkroom_offline.npz")
    n, H, permuted = (int(x) for x in g[f"{tag}/cfg"])
    _, m = ref_model("darkroom")
    trajs = []
    for i in range(n):
        t = {k: g[f"{tag}/{k}"][i] for k in ("context_states", "context_actions", "context_next_states",
                                              "context_rewards", "goal")}
        if permuted:
            t["perm_index"] = int(g[f"{tag}/perm_index"][i])
        trajs.append(t)
    u = g[f"{tag}/u"]
    res = eval_darkroom.offline(trajs, m, n_eval=n, H=H, dim=10, permuted=bool(permuted), uniforms=u)
    assert np.array_equal(res["Opt"], g[f"{tag}/opt_returns"])
    assert np.array_equal(res["Learner"], g[f"{tag}/lnr_rewards"].sum(-1))
    assert np.array_equal(res["Learner (greedy)"], g[f"{tag}/greedy_rewards"].sum(-1))
    envs = [DarkroomEnvPermuted(10, t["perm_index"], H) if permuted else DarkroomEnv(10, t["goal"], H)
            for t in trajs]
    vec = DarkroomEnvVec(envs)
    dev = dpt_hip.device()
    ctx = (torch.tensor(g[f"{tag}/context_states"], dtype=torch.float32, device=dev),
           torch.tensor(g[f"{tag}/context_actions"], dtype=torch.float32, device=dev),
           torch.tensor(g[f"{tag}/context_next_states"], dtype=torch.float32, device=dev),
           torch.tensor(g[f"{tag}/context_rewards"], dtype=torch.float32, device=dev))
    for sample, key in ((True, "lnr_rewards"), (False, "greedy_rewards")):
        ctrl = DarkroomTransformerController(m, batch_size=n, sample=sample)
        ctrl.uniforms = lambda k: u[k]
        _, _, _, er = eval_darkroom._episode_device(m.device_model(), ctrl, vec, ctx, H)
        assert np.array_equal(er.cpu().numpy(), g[f"{tag}/{key}"]), key


def test_training_mode_no_grad_test_loss_loop():
    """train.py:265-278 computes its test loss with the model in training mode under no_grad:
    that gives the reference's predictions (test=False, preds[:, 1:], net.py:60).  The training
    step (grad enabled) takes the HIP training path and returns the same predictions; its
    backward fills .grad for a model whose parameters live on the host, as the reference's
    does before `.to(device)` (the kernels get device copies; the gradients come back to the
    parameters' device)."""
    g, m = ref_model("bandit5")
    m.test = False
    b = {"query_states": torch.from_numpy(g["T8/query"]).float(), "zeros": torch.zeros(16, 7),
         "context_states": torch.from_numpy(g["T8/cs"]).float(), "context_actions": torch.from_numpy(g["T8/ca"]).float(),
         "context_next_states": torch.from_numpy(g["T8/cn"]).float(),
         "context_rewards": torch.from_numpy(g["T8/cr"]).float()}
    ref = g["T8/preds_train"]
    m.train()
    with torch.no_grad():
        out = m(b).cpu().numpy()
    assert out.shape == ref.shape
    assert (np.abs(out - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all()
    pred = m(b)
    assert pred.requires_grad
    assert (np.abs(pred.detach().cpu().numpy() - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all()
    pred.sum().backward()
    grads = [p.grad for n, p in m.named_parameters() if not n.endswith("wte.weight")]
    assert all(gr is not None and gr.device.type == "cpu" and torch.isfinite(gr).all() for gr in grads)


@pytest.mark.parametrize("A,H,C", [(5, 500, 0), (20, 300, 0), (7, 40, 150), (3, 30, 0)])
def test_policy_wave_kernel_vs_oracle(A, H, C):
    """dpt_rollout_policy (one 64-lane workgroup per task, context in LDS, per-arm pairwise sums split
    over lanes) against the float64 numpy oracle's classical controllers (oracle/dpt_oracle.py
    policy_action: ctrls/ctrl_bandit.py:22-380) on the same injected draws, at the shapes the retired
    lane-per-task kernel was compared at: Opt, Emp (online and offline), UCB, LCB and Thompson
    (sampled posterior), Gaussian and -- for UCB -- Bernoulli rewards, with and without a prefix
    context.  Actions, rewards and arm values bit-identical.  LinUCB and the Thompson 100-draw vote
    are pinned by the reference's own recorded runs (test_linucb_kernel_and_drop_in at lin_d 2..8,
    test_linear_offline_and_graph_match_reference): numpy's BLAS on this host may round LinUCB
    differently from the host those were recorded on (LinUCB orders)."""
    import dpt_hip
    from oracle import dpt_oracle as O
    rs = np.random.RandomState(A * 1000 + H + C)
    N = 48
    means = rs.uniform(0, 1, (N, A))
    ctx, octx = {}, {}
    if C:
        ca, cr = rs.randint(0, A, (N, C)).astype(np.int32), rs.normal(0.5, 0.5, (N, C))
        ctx = dict(ctx_actions=ca, ctx_rewards=cr)
        octx = dict(ctx_actions=ca.astype(np.int64), ctx_rewards=cr)
    ts = dict(std=0.3, prior_mean=0.5, prior_var=1 / 12.0)
    cases = [("opt", dpt_hip.POLICY_OPT, {}, {}),
             ("emp", dpt_hip.POLICY_EMP, dict(online=True), dict(online=True)),
             ("emp", dpt_hip.POLICY_EMP, dict(online=False), dict(online=False)),
             ("ucb", dpt_hip.POLICY_UCB, dict(c=1.0), dict(c=1.0)),
             ("lcb", dpt_hip.POLICY_LCB, dict(c=0.8), dict(c=0.8)),
             ("thompson", dpt_hip.POLICY_THOMPSON, dict(ts_std=0.3, ts_prior_mean=0.5, ts_prior_var=1 / 12.0),
              dict(ts=ts))]
    for name, pol, kw, okw in cases:
        for bern in ((False, True) if name == "ucb" else (False,)):
            g = rs.uniform(size=(H, N)) if bern else rs.normal(size=(H, N))
            pn = rs.normal(size=(H, N, A)) if name == "thompson" else None
            bt = dpt_hip.BANDIT_BERNOULLI if bern else dpt_hip.BANDIT_GAUSSIAN
            o = dpt_hip.rollout_policy(pol, means, H, 0.3, bandit_type=bt, noise=g, policy_noise=pn, **ctx, **kw)
            got = {k: o[k].cpu().numpy() for k in ("actions", "rewards", "arm_value")}
            if name == "opt":  # OptPolicy: the optimal arm every step (ctrl_bandit.py:22-38)
                acts = np.repeat(means.argmax(1)[:, None], H, 1)
                rew = np.stack([(O.bernoulli_reward(means, acts[:, h], g[h]) if bern
                                 else O.bandit_reward(means, acts[:, h], g[h], 0.3)) for h in range(H)], 1)
                ref = dict(actions=acts, rewards=rew, cum_means=np.stack([O.arm_value(means, acts[:, h])
                                                                          for h in range(H)]))
            else:
                ref = O.bandit_policy_rollout(name, means, H, 0.3, g, bernoulli=bern, ts_g=pn, **octx, **okw)
            assert np.array_equal(got["actions"], ref["actions"]), (name, kw, bern)
            assert np.array_equal(got["rewards"], ref["rewards"]), (name, kw, bern)
            assert np.array_equal(got["arm_value"].T, ref["cum_means"]), (name, kw, bern)


def test_policy_lane_kernel_retired():
    """DPT_TUNE_POLICY_WAVE accepts only the wave kernel since round 6; dpt_policy_workspace_numel is
    0 (the contexts live in LDS) and a null workspace is accepted."""
    import ctypes
    import dpt_hip
    from dpt_hip import _lib
    with pytest.raises(NotImplementedError):
        _lib.call("dpt_tuning_set", _lib.TUNE_POLICY_WAVE, 0)
    _lib.call("dpt_tuning_set", _lib.TUNE_POLICY_WAVE, 1)
    n = ctypes.c_int64(-1)
    _lib.call("dpt_policy_workspace_numel", 4096, 20, 1000, ctypes.byref(n))
    assert n.value == 0
    o = dpt_hip.rollout_policy(dpt_hip.POLICY_UCB, np.random.RandomState(0).uniform(0, 1, (8, 5)), 20, 0.3)
    assert o["actions"].shape == (8, 20)
