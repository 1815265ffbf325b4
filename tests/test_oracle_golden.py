"""Pin the CPU oracle (oracle/dpt_oracle.py) against vectors recorded from the reference."""
import numpy as np
import pytest

from conftest import golden
from oracle import dpt_oracle as O


def weights(name):
    g = golden(f"forward_{name}.npz")
    w = {k[2:]: v for k, v in g.items() if k.startswith("w/")}
    return g, O.split_weights(w, int(g["cfg"][3]))


def test_bandit_transit_bit_exact():
    g = golden("bandit_transit.npz")
    for var in (0.0, 0.3, 1.0):
        r = O.bandit_reward(g["means"], g["action"], g[f"g_var{var}"], var)
        assert np.array_equal(r.view(np.int64), g[f"reward_var{var}"].view(np.int64))
    assert np.array_equal(O.arm_value(g["means"], g["action"]), g["arm_value"])
    assert np.array_equal(np.argmax(g["means"], 1), g["opt_index"])
    lm = O.linear_means(g["lin_arms"], g["lin_theta"])
    assert np.array_equal(lm, g["lin_means"])
    assert np.array_equal(np.argmax(lm, 1), g["lin_opt"])


def test_darkroom_exhaustive_table():
    g = golden("darkroom_transit.npz")
    st = g["states"]
    for gi in range(100):
        goal = np.broadcast_to(st[gi], st.shape)
        assert np.array_equal(O.darkroom_opt_action(st, goal), g["opt_action"][gi])
        for a in range(5):
            ns, r = O.darkroom_transit(st, np.full(100, a), goal)
            assert np.array_equal(ns, g["next_state"][gi, a])
            assert np.array_equal(r, g["reward"][gi, a])
    perms = O.perm_table()
    assert np.array_equal(perms, g["perms"])
    goal = np.full((100, 2), 9)
    for pi in range(120):
        perm = np.broadcast_to(perms[pi], (100, 5))
        assert np.array_equal(O.darkroom_opt_action(st, goal, perm), g["perm_opt_action"][pi])
        for a in range(5):
            ns, r = O.darkroom_transit(st, np.full(100, a), goal, perm=perm)
            assert np.array_equal(ns, g["perm_next_state"][pi, a])
            assert np.array_equal(r, g["perm_reward"][pi, a])


@pytest.mark.parametrize("name", ["bandit5", "darkroom", "linear20"])
def test_forward_logits_within_1e5(name):
    g, W = weights(name)
    Ts = sorted({int(k.split("/")[0][1:]) for k in g if k.startswith("T")})
    for T in Ts:
        args = [g[f"T{T}/{k}"] for k in ("query", "cs", "ca", "cn", "cr")]
        ref = g[f"T{T}/logits"]
        got = O.transformer_forward(W, *args)
        tol = 1e-5 * np.maximum(1.0, np.abs(ref))
        assert (np.abs(got - ref) <= tol).all(), (T, np.abs(got - ref).max())
        if T > 1:
            got_all = O.transformer_forward(W, *args, test=False)
            ref_all = g[f"T{T}/preds_train"]
            assert np.abs(got_all - ref_all).max() <= 1e-5 * max(1, np.abs(ref_all).max())


def test_selection_matches_reference_choice():
    g = golden("select.npz")
    for A in (5, 20):
        lg, u = g[f"A{A}/logits"], g[f"A{A}/u"]
        assert np.array_equal(O.select_actions(lg, u), g[f"A{A}/sampled"])
        assert np.array_equal(O.select_actions(lg, sample=False), g[f"A{A}/greedy"])


@pytest.mark.parametrize("tag", ["sample", "greedy", "var0"])
def test_bandit_rollout_matches_reference(tag):
    g = golden(f"rollout_bandit_{tag}.npz")
    _, W = weights("bandit5")
    n, H, A, sample = g["cfg"]
    out = O.bandit_online_rollout(W, g["means"], int(H), float(g["var"]), g["u"], g["g"], bool(sample))
    assert np.abs(out["logits"] - g["logits"]).max() <= 1e-5
    assert np.array_equal(out["actions"], g["ctx_actions"].argmax(-1))
    assert np.array_equal(out["cum_means"], g["cum_means"])
    assert np.array_equal(out["rewards"], g["ctx_rewards"])


def test_linear_rollout_matches_reference():
    g = golden("rollout_linear_sample.npz")
    _, W = weights("linear20")
    n, H, A, sample = g["cfg"]
    assert np.array_equal(O.linear_means(g["arms"], g["theta"]), g["means"])
    out = O.bandit_online_rollout(W, g["means"], int(H), float(g["var"]), g["u"], g["g"], True)
    assert np.array_equal(out["cum_means"], g["cum_means"])
    assert np.array_equal(out["rewards"], g["ctx_rewards"])


@pytest.mark.parametrize("tag", ["sample", "greedy", "permuted"])
def test_darkroom_rollout_matches_reference(tag):
    g = golden(f"rollout_darkroom_{tag}.npz")
    _, W = weights("darkroom")
    n, Heps, H, horizon, sample = (int(x) for x in g["cfg"])
    perm = None
    if tag == "permuted":
        perm = O.perm_table()[g["perm_index"]]
    out = O.darkroom_online_rollout(W, g["goals"], Heps, H, horizon, g["u"], bool(sample), perm)
    assert np.abs(out["logits"] - g["logits"]).max() <= 1e-5
    assert np.array_equal(out["returns"], g["returns"])


def test_regret_math():
    g = golden("regret_math.npz")
    out = O.regret_curves(g["opt"], g["lnr"])
    for k in ("subopt_mean", "subopt_sem", "regret_mean", "regret_sem"):
        np.testing.assert_allclose(out[k], g[k], rtol=1e-12, atol=1e-15)


def test_rollin_bandit():
    g = golden("rollin.npz")
    for i in range(6):
        xs, us, xps, rs = O.rollin_bandit(g[f"{i}/means"], float(g[f"{i}/cov"]), g[f"{i}/dirichlet"],
                                          g[f"{i}/rand_index"], g[f"{i}/u"], g[f"{i}/g"], 0.3)
        assert np.array_equal(us, g[f"{i}/us"])
        assert np.array_equal(rs, g[f"{i}/rs"])
        assert np.array_equal(xs, g[f"{i}/xs"]) and np.array_equal(xps, g[f"{i}/xps"])
    s, a, ns, r = (g[f"mdp/{k}"] for k in ("states", "actions", "next_states", "rewards"))
    ns2, r2 = O.darkroom_transit(s, a.argmax(-1), np.broadcast_to(g["mdp/goal"], s.shape))
    assert np.array_equal(ns2, ns) and np.array_equal(r2, r)


@pytest.mark.parametrize("name", ["emp", "ucb", "thomp"])
def test_baseline_rollouts(name):
    g = golden("baselines.npz")
    kw = dict(emp=dict(policy="emp", online=True), ucb=dict(policy="ucb", c=1.0),
              thomp=dict(policy="thompson", ts=dict(std=0.3, prior_mean=0.5, prior_var=1 / 12.0)))[name]
    if name == "thomp":
        kw["ts_g"] = g["thomp/policy_g"]
    H = g[f"{name}/g"].shape[0]
    out = O.bandit_policy_rollout(kw.pop("policy"), g["means"], H, 0.3, g[f"{name}/g"], **kw)
    assert np.array_equal(out["actions"], g[f"{name}/actions"])
    assert np.array_equal(out["rewards"], g[f"{name}/rewards"])
    assert np.array_equal(out["cum_means"], g[f"{name}/cum_means"])


def test_baseline_offline_and_linucb():
    g = golden("baselines.npz")
    ca, cr = g["off/ctx_actions"], g["off/ctx_rewards"]
    assert np.array_equal(O.policy_action("emp", ca, cr, 5, online=False), g["off/emp/actions"])
    assert np.array_equal(O.policy_action("lcb", ca, cr, 5, c=0.8), g["off/lcb/actions"])
    H = g["lin/g"].shape[0]
    out = O.bandit_policy_rollout("linucb", g["lin/means"], H, 0.3, g["lin/g"], c=1.0, arms=g["lin/arms"],
                                  first_u_idx=g["lin/first_action"])
    assert np.array_equal(out["actions"], g["lin/actions"])
    assert np.array_equal(out["cum_means"], g["lin/cum_means"])


def test_c1_collect_and_eval_match_reference():
    """BASELINE config 1 at its size (64 tasks, H=100, 5 arms, var 0.3): the reference's
    generate_bandit_histories and the DPT online eval with its regret curves."""
    g = golden("c1_bandit.npz")
    N, H, A = (int(x) for x in g["cfg"])
    for i in range(N):
        _, us, _, rs = O.rollin_bandit(g["collect/means"][i], g["collect/cov"][i], g["collect/dirichlet"][i],
                                       g["collect/rand_index"][i], g["collect/u"][i], g["collect/g"][i], 0.3)
        assert np.array_equal(us.argmax(-1), g["collect/actions"][i]), i
        assert np.array_equal(rs, g["collect/rewards"][i]), i
    assert np.array_equal(g["collect/optimal_action"].argmax(-1), g["collect/means"].argmax(-1))
    _, W = weights("bandit5")
    out = O.bandit_online_rollout(W, g["eval/means"], H, float(g["var"]), g["eval/u"], g["eval/g"], True)
    assert np.array_equal(out["actions"], g["eval/actions"])
    assert np.array_equal(out["cum_means"], g["eval/cum_means"])
    assert np.array_equal(out["rewards"], g["eval/rewards"])
    opt = np.repeat(g["eval/means"].max(1, keepdims=True), H, axis=1)
    st = O.regret_curves(opt, g["eval/cum_means"].T)
    for k in ("subopt_mean", "subopt_sem", "regret_mean", "regret_sem"):
        np.testing.assert_allclose(st[k], g[f"eval/{k}"], rtol=1e-12, atol=1e-15)


def test_gpu_bandit_env_rewards_bit_exact():
    g = golden("gpu_bandit_env.npz")
    for var in (0.3, 1.0):
        for t in range(3):
            r = O.gpu_bandit_reward_f32(g[f"var{var}/means"], g[f"var{var}/actions"][t], g[f"var{var}/g"][t], var)
            assert r.dtype == np.float32
            assert np.array_equal(r.view(np.int32), g[f"var{var}/rewards"][t].view(np.int32)), (var, t)
        assert g[f"var{var}/done"][-1].all() and not g[f"var{var}/done"][:-1].any()


def test_linear_thompson_rollin_matches_reference():
    g = golden("linear_thompson.npz")
    H = g["g"].shape[0]
    assert np.array_equal(O.linear_means(g["arms"], g["theta"]), g["means"])
    out = O.bandit_policy_rollout("thompson", g["means"], H, float(g["var"]), g["g"],
                                  ts=dict(std=float(g["var"]), prior_mean=0.0, prior_var=1.0), ts_g=g["policy_g"])
    assert np.array_equal(out["actions"], g["context_actions"].argmax(-1))
    assert np.array_equal(out["rewards"], g["context_rewards"])


@pytest.mark.parametrize("tag", ["plain", "permuted"])
def test_darkroom_offline_matches_reference(tag):
    g = golden("darkroom_offline.npz")
    _, W = weights("darkroom")
    n, H, permuted = (int(x) for x in g[f"{tag}/cfg"])
    perm = O.perm_table()[g[f"{tag}/perm_index"]] if permuted else None
    goals = g[f"{tag}/goal"]
    ctx = (g[f"{tag}/context_states"].astype(np.float64), g[f"{tag}/context_actions"],
           g[f"{tag}/context_next_states"].astype(np.float64), g[f"{tag}/context_rewards"][..., None].astype(np.float64))
    assert np.array_equal(O.darkroom_opt_returns(goals, H, perm), g[f"{tag}/opt_returns"])
    greedy = O.darkroom_offline_episode(W, goals, ctx, H, None, sample=False, perm=perm)
    assert np.array_equal(greedy, g[f"{tag}/greedy_rewards"])
    lnr = O.darkroom_offline_episode(W, goals, ctx, H, g[f"{tag}/u"], sample=True, perm=perm)
    assert np.array_equal(lnr, g[f"{tag}/lnr_rewards"])


@pytest.mark.parametrize("tag", ["sample", "greedy", "permuted"])
def test_c_darkroom_oracle_matches_reference(tag):
    """The float64 C restatement of the DarkRoom online eval (oracle/dpt_oracle.c, the full-size
    checker of the GPU tests) against the reference's recorded rollouts, memo on and off."""
    import torch
    from oracle import c_oracle
    import dpt_hip
    g = golden(f"rollout_darkroom_{tag}.npz")
    fw, _ = weights("darkroom")
    n, Heps, H, horizon, sample = (int(x) for x in g["cfg"])
    sd = {k[2:]: torch.from_numpy(v) for k, v in fw.items() if k.startswith("w/")}
    blob = dpt_hip.pack_weights(sd, 4).numpy()
    perm = O.perm_table()[g["perm_index"]] if tag == "permuted" else None
    u = g["u"].reshape(Heps * horizon, n) if sample else None
    outs = [c_oracle.darkroom_rollout(blob, 4, 404, g["goals"], Heps, horizon, H // horizon, u, bool(sample), perm,
                                      memo=memo, threads=2, want_logits=True) for memo in (False, True)]
    for o in outs:
        assert np.abs(o["logits"] - g["logits"]).max() <= 1e-5
        assert np.array_equal(o["returns"], g["returns"])
    assert np.array_equal(outs[0]["actions"], outs[1]["actions"])


@pytest.mark.parametrize("dim,R,horizon", [(10, 2, 30), (12, 1, 37), (11, 3, 13)])
def test_c_darkroom_oracle_equals_numpy_oracle(dim, R, horizon):
    """The vectorised float64 C DarkRoom forward (phase by phase over the tokens, 4-row register
    blocks, transposed keys padded to 16, libmvec exp) against the plain numpy float64 restatement
    (oracle/dpt_oracle.py darkroom_online_rollout) at windows that are not multiples of 4 or 16, grids
    over 10 x 10 and several context episodes: logits within 1e-6 (float32-rounded float64 logits), the
    same actions and returns."""
    import torch
    from oracle import c_oracle
    import dpt_hip
    fw, W = weights("darkroom")
    sd = {k[2:]: torch.from_numpy(v) for k, v in fw.items() if k.startswith("w/")}
    blob = dpt_hip.pack_weights(sd, 4).numpy()
    rs = np.random.RandomState(dim * 10 + R)
    N, Heps = 5, R + 2
    goals = rs.randint(0, dim, (N, 2))
    u = rs.uniform(size=(Heps, horizon, N))
    ref = O.darkroom_online_rollout(W, goals, Heps, R * horizon, horizon, u, True, dim=dim)
    got = c_oracle.darkroom_rollout(blob, 4, 404, goals, Heps, horizon, R, u.reshape(Heps * horizon, N), True,
                                    dim=dim, threads=2, want_logits=True)
    assert np.abs(got["logits"] - ref["logits"]).max() <= 1e-6
    assert np.array_equal(got["actions"], ref["actions"])
    assert np.array_equal(got["returns"], ref["returns"])


def _bandit_cases():
    """(fixture, weights, means, H, var, u, g, sample, ref actions, ref cum_means, ref rewards, ref logits)
    of every recorded reference bandit rollout (evals/eval_bandit.py:56-103 with the DPT controller)."""
    for tag in ("sample", "greedy", "var0"):
        yield f"rollout_bandit_{tag}", "bandit5"
    yield "rollout_linear_sample", "linear20"
    yield "c1_bandit", "bandit5"


@pytest.mark.parametrize("fix,wname", list(_bandit_cases()))
@pytest.mark.parametrize("mode", ["f32", "f64"])
def test_c_bandit_oracle_matches_reference(fix, wname, mode):
    """The C restatement of the bandit online rollout (oracle/dpt_oracle.c: the fp32 CPU baseline
    and the float64 full-size checker of the GPU tests) against the reference's recorded rollouts
    with its draws injected: actions, rewards and cum_means exactly, logits within 1e-5.  The
    float64 form is also checked in its re-forward-every-step (reference) shape."""
    import torch
    from oracle import c_oracle
    import dpt_hip
    g = golden(f"{fix}.npz")
    fw, _ = weights(wname)
    Hw, _, A, L, _ = (int(x) for x in fw["cfg"])
    sd = {k[2:]: torch.from_numpy(v) for k, v in fw.items() if k.startswith("w/")}
    blob = dpt_hip.pack_weights(sd, L).numpy()
    npos = 4 * (1 + Hw)
    if fix == "c1_bandit":
        means, u, gg = g["eval/means"], g["eval/u"], g["eval/g"]
        H, sample = int(g["cfg"][1]), True
        ref_a, ref_cm, ref_r, ref_lg = g["eval/actions"], g["eval/cum_means"], g["eval/rewards"], None
    else:
        means, u, gg = g["means"], g["u"], g["g"]
        _, H, _, sample = (int(x) for x in g["cfg"])
        ref_a, ref_cm, ref_r, ref_lg = g["ctx_actions"].argmax(-1), g["cum_means"], g["ctx_rewards"], g["logits"]
    var = float(g["var"])
    runs = []
    if mode == "f32":
        runs.append(c_oracle.bandit_rollout(blob, L, A, npos, means, H, var, u, gg, bool(sample), False, 2,
                                            want_logits=True))
    else:
        for rec in (False, True):
            runs.append(c_oracle.bandit_rollout_f64(blob, L, A, npos, means, H, var, u, gg, bool(sample), rec, 2,
                                                    want_logits=True))
        assert np.array_equal(runs[0]["logits"], runs[1]["logits"])  # decode == re-forward, bit for bit
    for o in runs:
        if ref_lg is not None:
            assert np.abs(o["logits"] - ref_lg).max() <= 1e-5
        assert np.array_equal(o["actions"], ref_a)
        assert np.array_equal(o["rewards"], ref_r)
        assert np.array_equal(o["cum_means"], ref_cm)


@pytest.mark.parametrize("name", ["darkroom", "bandit5"])
def test_torch_oracle_gradients_match_reference(name):
    """oracle/dpt_oracle_torch.py (float64 autograd of the restated forward, the checker of the
    HIP training kernels) against the gradients recorded from the reference's train.py loss."""
    from oracle import dpt_oracle_torch as OT
    g = golden("train_grads.npz")
    fw = golden(f"forward_{name}.npz")
    H, sd, A, L, _ = (int(x) for x in fw["cfg"])
    w = {k[2:]: v for k, v in fw.items() if k.startswith("w/")}
    batch = {k: g[f"{name}/{k}"] for k in ("query_states", "context_states", "context_actions",
                                           "context_next_states", "context_rewards", "optimal_actions")}
    loss, preds, gr = OT.grads(w, batch, L, sd, A)
    assert abs(loss - float(g[f"{name}/f64/loss"])) <= 1e-10 * abs(loss)
    assert np.abs(preds - g[f"{name}/f64/preds"]).max() <= 1e-12
    for k, v in gr.items():
        ref = g[f"{name}/f64/grad/{k}"]
        got = v[:ref.shape[0]] if k.endswith("wpe.weight") else v
        if k.endswith("wpe.weight"):
            assert not v[ref.shape[0]:].any()
        assert np.abs(got - ref).max() <= 1e-10 * max(1e-30, np.abs(ref).max()), k


@pytest.mark.parametrize("fix", ["linucb_d4", "linucb_long", "linucb_dims:3", "linucb_dims:5", "linucb_dims:6",
                                 "linucb_dims:8"])
def test_linucb_matches_reference(fix):
    """LinUCB with lin_d = 4, lin_d = 2 over 800 steps, and lin_d 3 / 5 / 6 / 8 over 100 steps
    (np.linalg.inv in the oracle, as in the reference)."""
    g = golden_lin(fix)
    H = g["g"].shape[0]
    out = O.bandit_policy_rollout("linucb", g["means"], H, 0.3, g["g"], c=1.0, arms=g["arms"],
                                  first_u_idx=g["first_action"])
    assert np.array_equal(out["actions"], g["actions"])
    assert np.array_equal(out["cum_means"], g["cum_means"])


def golden_lin(fix):
    """a LinUCB fixture: "name" or "linucb_dims:<lin_d>" (one width of the multi-width file)"""
    if ":" not in fix:
        return golden(f"{fix}.npz")
    name, d = fix.split(":")
    g = golden(f"{name}.npz")
    return {k.split("/", 1)[1]: g[k] for k in g if k.startswith(f"d{d}/")}


@pytest.mark.parametrize("case", [0, 1])
def test_torch_oracle_dropout_matches_reference(case):
    """Training-mode dropout (GPT2Config embd/attn/resid_pdrop, models/net.py:30-32): the
    float64 oracle with the kernels' Philox masks (tests/philox_np.dropout_keep) against the
    reference model run with the same masks injected at its dropout calls
    (tests/golden/train_dropout.npz; gen_golden.py train_dropout checks each call's site by order
    and shape) -- pins the placement of every mask: embedding sum, attention probabilities,
    c_proj and mlp.c_proj outputs."""
    import torch
    from oracle import dpt_oracle_torch as OT
    from philox_np import dropout_keep
    g = golden("train_dropout.npz")
    fw = golden("forward_bandit5.npz")
    H, sd, A, L, E = (int(x) for x in fw["cfg"])
    w = {k[2:]: v for k, v in fw.items() if k.startswith("w/")}
    pre = f"c{case}/"
    batch = {k: g[pre + k] for k in ("query_states", "context_states", "context_actions", "context_next_states",
                                     "context_rewards", "optimal_actions")}
    B, T = batch["context_states"].shape[0], batch["context_states"].shape[1] + 1
    p, seed = float(g[pre + "p"]), int(g[pre + "seed"])

    def drop(site):
        shape = (B, T, T) if site % 3 == 1 else (B, T, E)
        return torch.from_numpy(dropout_keep(seed, p, site, shape))
    loss, preds, gr = OT.grads(w, batch, L, sd, A, drop=drop)
    assert abs(loss - float(g[pre + "loss"])) <= 1e-10 * abs(loss)
    assert np.abs(preds - g[pre + "preds"]).max() <= 1e-12
    for k, v in gr.items():
        ref = g[pre + "grad/" + k]
        got = v[:ref.shape[0]] if k.endswith("wpe.weight") else v
        assert np.abs(got - ref).max() <= 1e-10 * max(1e-30, np.abs(ref).max()), k
    # the masks drop about p of the elements (a loose sanity bar on the threshold)
    k0 = dropout_keep(seed, p, 0, (64, 1024))
    assert abs((k0 == 0).mean() - p) < 0.01
