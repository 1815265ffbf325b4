"""Parity of the HIP kernels (through the C ABI) against reference golden vectors and the oracle.

Bars: bit-exact for env transitions, indices, rewards and arm values; logits
within 1e-5 * max(1, |x|) (BASELINE.json north_star); sampled actions exact
wherever the uniform is further than 1e-5 from a cdf edge (flagged otherwise).
"""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import dpt_oracle as O
import philox_np

pytestmark = pytest.mark.gpu

LOGIT_TOL = 1e-5


def dh():
    import dpt_hip
    dpt_hip.device()
    return dpt_hip


def model_from_golden(name):
    import dpt_hip
    g = golden(f"forward_{name}.npz")
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")}
    H, sd, A, L, E = (int(x) for x in g["cfg"])
    m = dpt_hip.DeviceModel(w, L, sd, A, 4 * (1 + H))
    W = O.split_weights({k: v.numpy() for k, v in w.items()}, L)
    return g, m, W


def assert_logits(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    err = np.abs(got - ref)
    assert (err <= LOGIT_TOL * np.maximum(1.0, np.abs(ref))).all(), err.max()


def test_bandit_step_bit_exact():
    d = dh()
    g = golden("bandit_transit.npz")
    for var in (0.0, 0.3, 1.0):
        r, v = d.bandit_step(g["means"], g["action"], var, noise=g[f"g_var{var}"])
        assert np.array_equal(r.cpu().numpy().view(np.int64), g[f"reward_var{var}"].view(np.int64))
        assert np.array_equal(v.cpu().numpy(), g["arm_value"])


def test_bandit_step_bernoulli_and_philox():
    d = dh()
    rs = np.random.RandomState(0)
    means = rs.uniform(0, 1, (1000, 5))
    a = rs.randint(0, 5, 1000)
    u = rs.uniform(size=1000)
    r, _ = d.bandit_step(means, a, 0.0, d.BANDIT_BERNOULLI, noise=u)
    assert np.array_equal(r.cpu().numpy(), O.bernoulli_reward(means, a, u))
    # Philox path: rewards equal the oracle fed with the draws the library reports
    seed, step = 1234567, 17
    r, _ = d.bandit_step(means, a, 0.3, seed=seed, counter=step, first_task=100)
    gdraw = d.draw(1, seed, step, 100, 1000, d.STREAM_REWARD).cpu().numpy()
    assert np.array_equal(r.cpu().numpy(), O.bandit_reward(means, a, gdraw, 0.3))
    np.testing.assert_allclose(gdraw, philox_np.normal(seed, step, np.arange(100, 1100), d.STREAM_REWARD),
                               rtol=1e-12, atol=1e-12)
    udraw = d.draw(0, seed, step, 5, 1000, d.STREAM_SELECT).cpu().numpy()
    assert np.array_equal(udraw, philox_np.uniform(seed, step, np.arange(5, 1005), d.STREAM_SELECT))
    assert 0.45 < udraw.mean() < 0.55 and abs(gdraw.mean()) < 0.1 and 0.9 < gdraw.std() < 1.1


def test_darkroom_exhaustive():
    d = dh()
    g = golden("darkroom_transit.npz")
    st = np.tile(g["states"], (100 * 5, 1))
    goals = np.repeat(g["states"], 100, axis=0)
    goals5 = np.repeat(goals[None], 5, 0).reshape(-1, 2)
    acts = np.repeat(np.arange(5), 100 * 100)
    # order (a, goal, state)
    ns, r = d.darkroom_step(st, acts, goals5)
    ref_ns = g["next_state"].transpose(1, 0, 2, 3).reshape(-1, 2)
    ref_r = g["reward"].transpose(1, 0, 2).reshape(-1)
    assert np.array_equal(ns.cpu().numpy(), ref_ns)
    assert np.array_equal(r.cpu().numpy(), ref_r)
    opt = d.darkroom_opt_action(np.tile(g["states"], (100, 1)), goals)
    assert np.array_equal(opt.cpu().numpy(), g["opt_action"].reshape(-1))
    # permuted: goal fixed at (9, 9)
    perms = g["perms"].astype(np.int32)
    st = np.tile(g["states"], (120 * 5, 1))
    pidx = np.repeat(np.tile(np.arange(120), 5), 100)
    acts = np.repeat(np.arange(5), 120 * 100)
    goal = np.full((len(st), 2), 9)
    ns, r = d.darkroom_step(st, acts, goal, perm=perms[pidx])
    assert np.array_equal(ns.cpu().numpy(), g["perm_next_state"].transpose(1, 0, 2, 3).reshape(-1, 2))
    assert np.array_equal(r.cpu().numpy(), g["perm_reward"].transpose(1, 0, 2).reshape(-1))
    st1 = np.tile(g["states"], (120, 1))
    opt = d.darkroom_opt_action(st1, np.full((len(st1), 2), 9), perm=perms[np.repeat(np.arange(120), 100)])
    assert np.array_equal(opt.cpu().numpy(), g["perm_opt_action"].reshape(-1))


def test_select_action_matches_reference():
    d = dh()
    g = golden("select.npz")
    for A in (5, 20):
        lg, u = g[f"A{A}/logits"], g[f"A{A}/u"]
        got = d.select_action(lg, True, uniforms=u).cpu().numpy()
        margin = O.boundary_margin(O.softmax_f32(lg), u)
        ok = margin > 1e-5
        assert np.array_equal(got[ok], g[f"A{A}/sampled"][ok]), np.nonzero(got != g[f"A{A}/sampled"])
        assert np.array_equal(d.select_action(lg, False).cpu().numpy(), g[f"A{A}/greedy"])
    # temperature path (ctrl_darkroom.py:51 divides by temp)
    lg = g["A5/logits"]
    u = g["A5/u"]
    got = d.select_action(lg, True, temp=0.5, uniforms=u).cpu().numpy()
    ref = O.select_actions(lg, u, True, temp=0.5)
    ok = O.boundary_margin(O.softmax_f32(lg, 0.5), u) > 1e-5
    assert np.array_equal(got[ok], ref[ok])


def test_select_fast_path_equals_fp64_cdf():
    """select_fast (fp32 cdf, exact fp64 cdf within 2^-15 of an edge; the rollouts' selection)
    against the fp64-only path on adversarial draws: uniforms placed 1e-9 .. 1e-3 either side of
    every cdf edge, logit spreads up to 60, temperature 1 and 0.5, NaN rows.  Bit-identical."""
    d = dh()
    rs = np.random.RandomState(11)
    for A in (5, 20):
        for spread in (0.1, 3.0, 20.0, 60.0):
            lg = (rs.randn(4096, A) * spread).astype(np.float32)
            lg[::97] = lg[::97, :1]  # ties
            for temp in (1.0, 0.5):
                cdf = np.cumsum(O.softmax_f32(lg, temp).astype(np.float64), -1)
                cdf /= cdf[:, -1:]
                k = rs.randint(0, A - 1, 4096)
                delta = rs.choice([1e-9, 1e-7, 1e-6, 1e-5, 3e-5, 1e-4, 1e-3], 4096) * rs.choice([-1, 1], 4096)
                u = np.clip(cdf[np.arange(4096), k] + delta, 0.0, np.nextafter(1.0, 0.0))
                u[::5] = rs.uniform(0, 1, u[::5].shape)
                lgn = lg.copy()
                lgn[::211, 1] = np.nan
                for logits in (lgn, lg):
                    d.set_select_fast(False)
                    ref = d.select_action(logits, True, temp=temp, uniforms=u).cpu().numpy()
                    d.set_select_fast(True)
                    got = d.select_action(logits, True, temp=temp, uniforms=u).cpu().numpy()
                    assert np.array_equal(got, ref), (A, spread, temp, np.nonzero(got != ref)[0][:10])
                # and the reference's own selection away from the edges (numpy's expf is not
                # correctly rounded, so nearer than 1e-5 only the device paths are compared)
                ok = O.boundary_margin(O.softmax_f32(lg, temp), u) > 1e-5
                assert np.array_equal(got[ok], O.select_actions(lg, u, True, temp=temp)[ok])
    d.set_select_fast(True)


@pytest.mark.parametrize("name", ["bandit5", "darkroom", "linear20"])
def test_forward_window_logits(name):
    g, m, W = model_from_golden(name)
    Ts = sorted({int(k.split("/")[0][1:]) for k in g if k.startswith("T")})
    for T in Ts:
        q, cs, ca, cn, cr = (g[f"T{T}/{k}"] for k in ("query", "cs", "ca", "cn", "cr"))
        C = T - 1
        args = (q,) if C == 0 else (q, cs, ca, cn, cr)
        out = m.forward_window(*args).cpu().numpy()
        assert_logits(out, g[f"T{T}/logits"])
        if C >= 1:
            allp = m.forward_window(q, cs, ca, cn, cr, out_mode=1).cpu().numpy()
            assert_logits(allp, g[f"T{T}/preds_train"])


def test_decode_steps_equal_window():
    import dpt_hip
    g, m, W = model_from_golden("bandit5")
    q, cs, ca, cn, cr = (g[f"T101/{k}"] for k in ("query", "cs", "ca", "cn", "cr"))
    N, C = cs.shape[:2]
    seq = O.pack_tokens(q, cs, ca, cn, cr, 5, 1).astype(np.float32)
    kv = torch.empty(m.kv_numel(N, C + 1), dtype=torch.float32, device=dpt_hip.device())
    for p in range(C + 1):
        lg = m.decode_step(kv, C + 1, p, seq[:, p]).cpu().numpy()
    try:  # the position-by-position window path is the same arithmetic as the decode steps
        dpt_hip.set_prefill(False)
        win = m.forward_window(q, cs, ca, cn, cr).cpu().numpy()
    finally:
        dpt_hip.set_prefill(True)
    assert np.array_equal(lg, win)
    assert_logits(lg, g["T101/logits"])
    assert_logits(m.forward_window(q, cs, ca, cn, cr).cpu().numpy(), lg)  # MFMA prefill: summation order differs


@pytest.mark.parametrize("tag", ["sample", "greedy", "var0"])
def test_rollout_bandit_matches_reference(tag):
    r = golden(f"rollout_bandit_{tag}.npz")
    _, m, W = model_from_golden("bandit5")
    n, H, A, sample = (int(x) for x in r["cfg"])
    out = m.rollout_bandit(r["means"], H, float(r["var"]), bool(sample), uniforms=r["u"] if sample else None,
                           noise=r["g"], want_logits=True)
    assert_logits(out["logits"].cpu().numpy(), r["logits"])
    assert np.array_equal(out["actions"].cpu().numpy(), r["ctx_actions"].argmax(-1))
    assert np.array_equal(out["rewards"].cpu().numpy(), r["ctx_rewards"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, r["cum_means"])


def test_rollout_linear_matches_reference():
    r = golden("rollout_linear_sample.npz")
    _, m, W = model_from_golden("linear20")
    n, H, A, sample = (int(x) for x in r["cfg"])
    out = m.rollout_bandit(r["means"], H, float(r["var"]), True, uniforms=r["u"], noise=r["g"],
                           want_logits=True)
    assert_logits(out["logits"].cpu().numpy(), r["logits"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, r["cum_means"])


def test_rollout_philox_vs_oracle_and_sharding():
    """Philox draws: the device rollout equals the oracle fed the same draws, and
    splitting the tasks over 'ranks' (first_task offsets) changes nothing."""
    d = dh()
    _, m, W = model_from_golden("bandit5")
    rs = np.random.RandomState(5)
    N, H, seed = 24, 20, 987654321
    means = rs.uniform(0, 1, (N, 5))
    full = m.rollout_bandit(means, H, 0.3, True, seed=seed)
    u = np.stack([philox_np.uniform(seed, h, np.arange(N), d.STREAM_SELECT) for h in range(H)])
    g = np.stack([d.draw(1, seed, h, 0, N, d.STREAM_REWARD).cpu().numpy() for h in range(H)])
    ref = O.bandit_online_rollout(W, means, H, 0.3, u, g, True)
    acts = full["actions"].cpu().numpy()
    assert np.array_equal(acts, ref["actions"])
    assert np.array_equal(full["arm_value"].cpu().numpy().T, ref["cum_means"])
    a = m.rollout_bandit(means[:10], H, 0.3, True, seed=seed, first_task=0)
    b = m.rollout_bandit(means[10:], H, 0.3, True, seed=seed, first_task=10)
    assert np.array_equal(np.concatenate([a["actions"].cpu().numpy(), b["actions"].cpu().numpy()]), acts)
    assert np.array_equal(np.concatenate([a["rewards"].cpu().numpy(), b["rewards"].cpu().numpy()]),
                          full["rewards"].cpu().numpy())


def test_rollout_large_properties():
    """Full-size invariants at N=4096 (config 2 width) on a shorter horizon:
    determinism, arm_value == means[action], rewards == means[a] + var*g."""
    d = dh()
    _, m, _ = model_from_golden("bandit5")
    rs = np.random.RandomState(1)
    N, H = 4096, 48
    means = rs.uniform(0, 1, (N, 5))
    o1 = m.rollout_bandit(means, H, 0.3, True, seed=42)
    o2 = m.rollout_bandit(means, H, 0.3, True, seed=42)
    a = o1["actions"].cpu().numpy()
    assert np.array_equal(a, o2["actions"].cpu().numpy())
    assert a.min() >= 0 and a.max() < 5
    av = o1["arm_value"].cpu().numpy()
    assert np.array_equal(av, means[np.arange(N)[:, None], a])
    g = np.stack([d.draw(1, 42, h, 0, N, d.STREAM_REWARD).cpu().numpy() for h in range(H)], 1)
    assert np.array_equal(o1["rewards"].cpu().numpy(), av + (0.0 + 0.3 * g))
    # partial tile (N not a multiple of 16) behaves like the full run on its prefix
    o3 = m.rollout_bandit(means[:1000], H, 0.3, True, seed=42)
    assert np.array_equal(o3["actions"].cpu().numpy(), a[:1000])


def test_decode_tiles_bit_identical():
    """TILE 8 (two workgroups per CU) and TILE 16 give bit-identical rollouts and windows
    (block 0 on the vector ALUs at both tiles: the matrix-core block 0 is a tile-8 path)."""
    import dpt_hip
    _, m, _ = model_from_golden("bandit5")
    rs = np.random.RandomState(9)
    means = rs.uniform(0, 1, (100, 5))
    outs = []
    g, mw, _ = model_from_golden("darkroom")
    q, cs, ca, cn, cr = (g[f"T101/{k}"] for k in ("query", "cs", "ca", "cn", "cr"))
    try:
        dpt_hip.set_block0_mfma(False)
        for tile in (16, 8):
            dpt_hip.set_decode_tile(tile)
            o = m.rollout_bandit(means, 40, 0.3, True, seed=5, want_logits=True)
            w = mw.forward_window(q, cs, ca, cn, cr, out_mode=1)
            outs.append([o["actions"].cpu().numpy(), o["rewards"].cpu().numpy(), o["logits"].cpu().numpy(),
                         w.cpu().numpy()])
    finally:
        dpt_hip.set_decode_tile(8)  # the library defaults
        dpt_hip.set_block0_mfma(False)
    for a, b in zip(*outs):
        assert np.array_equal(a, b)
    assert_logits(outs[1][3], g["T101/preds_train"])


@pytest.mark.parametrize("N,H", [(100, 40), (1000, 130)])
def test_rollout_block0_mfma_matches_vector_path(N, H):
    """Block 0 on the matrix cores (l0_tiles / l0_merge, DPT_TUNE_BLOCK0_MFMA) against
    the one-wave-per-task vector path: same algebra, another fp32 summation order.  Per task, the
    per-step logits agree within the 1e-5 bar up to the first step whose sampled action differs
    (a uniform within rounding of a cdf edge), and such divergences are rare."""
    import dpt_hip
    _, m, _ = model_from_golden("bandit5")
    means = np.random.RandomState(13).uniform(0, 1, (N, 5))
    outs = []
    try:
        for on in (False, True):
            dpt_hip.set_block0_mfma(on)
            o = m.rollout_bandit(means, H, 0.3, True, seed=17, want_logits=True)
            outs.append((o["actions"].cpu().numpy(), o["logits"].cpu().numpy()))
    finally:
        dpt_hip.set_block0_mfma(False)
    (a0, l0), (a1, l1) = outs
    diff = a0 != a1
    first = np.where(diff.any(1), diff.argmax(1), H)  # first differing step per task
    assert (first < H).mean() <= 0.01
    for t in range(N):
        f = first[t]
        # logits of steps <= f were computed on identical contexts
        assert_logits(l1[: f + 1 if f < H else H, t], l0[: f + 1 if f < H else H, t])


def test_rollout_cache_budget_bit_identical():
    """DPT_TUNE_CACHE_BUDGET only moves the default/non-temporal split of the y stream: budgets of
    0, one chunk (block 1 only), four chunks (every block 64 positions, block 1 128) and everything
    give bit-identical rollouts."""
    import dpt_hip
    _, m, _ = model_from_golden("bandit5")
    N, H = 300, 150
    means = np.random.RandomState(11).uniform(0, 1, (N, 5))
    chunk = N * 32 * 4 * 64  # one 64-position stream chunk of one block, all tasks
    outs = []
    try:
        for budget in (0, chunk, 4 * chunk, 1 << 40):
            dpt_hip.set_cache_budget(budget)
            o = m.rollout_bandit(means, H, 0.3, True, seed=7, want_logits=True)
            outs.append([o[k].cpu().numpy() for k in ("actions", "rewards", "arm_value", "logits")])
    finally:
        dpt_hip.set_cache_budget(224 << 20)  # the library default
    for other in outs[1:]:
        for a, b in zip(outs[0], other):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("tag", ["sample", "greedy", "permuted"])
def test_rollout_darkroom_fused_matches_reference(tag):
    """dpt_rollout_darkroom against the reference's deploy_online_vec recorded with the same draws:
    per-step logits (1e-5) and per-episode returns (exact), incl. R=2 shift-append and permuted actions."""
    r = golden(f"rollout_darkroom_{tag}.npz")
    _, m, _ = model_from_golden("darkroom")
    n, Heps, H, horizon, sample = (int(x) for x in r["cfg"])
    perms = O.perm_table()[r["perm_index"]] if tag == "permuted" else None
    out = m.rollout_darkroom(r["goals"], Heps, horizon, H // horizon, perms=perms, sample=bool(sample),
                             uniforms=r["u"].reshape(-1, n), want_actions=True, want_logits=True)
    assert_logits(out["logits"].cpu().numpy(), r["logits"])
    assert np.array_equal(out["returns"].cpu().numpy(), r["returns"])


@pytest.mark.parametrize("Heps,horizon,R", [(3, 30, 2), (2, 127, 1), (3, 64, 2), (2, 255, 1)])
def test_rollout_darkroom_philox_vs_oracle(Heps, horizon, R):
    """Philox draws (the select stream of dpt_select_action) through the fused kernel equal the
    oracle fed the same uniforms; (2, 127, 1) is the largest window of the 4-wave kernel
    (1 + R*horizon = 128), (3, 64, 2) the smallest of the 8-wave one (129) and (2, 255, 1) its
    largest (256)."""
    d = dh()
    _, m, W = model_from_golden("darkroom")
    rs = np.random.RandomState(3)
    N, seed, ctr = 6, 1234567, 7
    goals = rs.randint(0, 10, (N, 2))
    out = m.rollout_darkroom(goals, Heps, horizon, R, seed=seed, counter=ctr, want_actions=True, want_logits=True)
    steps = Heps * horizon
    u = np.stack([philox_np.uniform(seed, ctr + k, np.arange(N), d.STREAM_SELECT) for k in range(steps)])
    ref = O.darkroom_online_rollout(W, goals, Heps, R * horizon, horizon, u.reshape(Heps, horizon, N), True)
    lg = out["logits"].cpu().numpy()
    margin = O.boundary_margin(O.softmax_f32(ref["logits"], 1.0), u)
    if (margin < 1e-5).any():  # a near-tie sample may legitimately flip: compare up to it
        k = int(np.argmax((margin < 1e-5).any(-1)))
        assert_logits(lg[:k + 1], ref["logits"][:k + 1])
        pytest.skip(f"near-tie draw at step {k}")
    assert_logits(lg, ref["logits"])
    assert np.array_equal(out["returns"].cpu().numpy(), ref["returns"])


def test_rollout_darkroom_large_properties():
    """Config-3 width (N=4096, window 101) on 2 episodes: deterministic, shard-invariant
    (first_task offsets), returns within [0, horizon]; greedy logits equal the window kernel's."""
    _, m, _ = model_from_golden("darkroom")
    goals = np.stack(np.unravel_index(np.arange(4096) % 100, (10, 10)), 1)
    o1 = m.rollout_darkroom(goals, 2, 100, 1, seed=11, want_actions=True)
    o2 = m.rollout_darkroom(goals, 2, 100, 1, seed=11, want_actions=True)
    a1, r1 = o1["actions"].cpu().numpy(), o1["returns"].cpu().numpy()
    assert np.array_equal(a1, o2["actions"].cpu().numpy()) and np.array_equal(r1, o2["returns"].cpu().numpy())
    assert r1.min() >= 0 and r1.max() <= 100 and a1.min() >= 0 and a1.max() < 5
    lo = m.rollout_darkroom(goals[:1000], 2, 100, 1, seed=11, want_actions=True)
    hi = m.rollout_darkroom(goals[1000:], 2, 100, 1, seed=11, first_task=1000, want_actions=True)
    assert np.array_equal(np.concatenate([lo["actions"].cpu().numpy(), hi["actions"].cpu().numpy()]), a1)
    # greedy episode 1 logits == the per-step window kernel on the recorded context
    og = m.rollout_darkroom(goals[:64], 2, 100, 1, sample=False, want_actions=True, want_logits=True)
    acts = og["actions"].cpu().numpy()
    st = np.zeros((64, 2), np.int64)
    cs, ca, cn, cr = [], [], [], []
    for t in range(100):
        ns, rr = O.darkroom_transit(st, acts[:, t], goals[:64])
        cs.append(st.copy()); ca.append(np.eye(5)[acts[:, t]]); cn.append(ns.copy()); cr.append(rr)
        st = ns
    ctx = [np.stack(x, 1).astype(np.float32) for x in (cs, ca, cn, cr)]
    st = np.zeros((64, 2), np.int64)
    lg = og["logits"].cpu().numpy()
    for t in range(100):
        w = m.forward_window(st.astype(np.float32), *ctx).cpu().numpy()
        assert_logits(lg[100 + t], w)
        ns, _ = O.darkroom_transit(st, acts[:, 100 + t], goals[:64])
        st = ns


@pytest.mark.parametrize("sample", [1, 0])
@pytest.mark.parametrize("permuted", [False, True])
def test_rollout_darkroom_memo_bit_identical(sample, permuted):
    """The per-episode logits memo (one window forward per distinct query state) changes nothing:
    actions, per-step logits and returns are bit-identical to one forward per step, and the
    forward counter equals the number of distinct (episode, state) pairs the trajectory visits.
    Greedy selection (sample=0) is where the memo-hit runs are longest; permuted actions go
    through the per-task action permutation of DarkroomEnvPermuted."""
    import dpt_hip
    import itertools
    _, m, _ = model_from_golden("darkroom")
    rs = np.random.RandomState(5 + 2 * sample + permuted)
    N, Heps, horizon, R = 512, 3, 100, 1
    goals = rs.randint(0, 10, (N, 2))
    perms = None
    if permuted:
        table = np.array(list(itertools.permutations(range(5))), np.int32)
        perms = table[rs.randint(0, len(table), N)]
    outs = []
    try:
        for memo in (False, True):
            dpt_hip.set_darkroom_memo(memo)
            o = m.rollout_darkroom(goals, Heps, horizon, R, perms=perms, sample=bool(sample), seed=21,
                                   want_actions=True, want_logits=True, want_forwards=True)
            outs.append({k: o[k].cpu().numpy() for k in ("actions", "logits", "returns", "forwards")})
    finally:
        dpt_hip.set_darkroom_memo(True)  # the library default
    off, on = outs
    for k in ("actions", "logits", "returns"):
        assert np.array_equal(off[k], on[k]), k
    assert (off["forwards"] == horizon).all()
    acts = on["actions"].reshape(N, Heps, horizon)
    distinct = np.zeros((N, Heps), np.int64)
    for e in range(Heps):
        st = np.zeros((N, 2), np.int64)
        seen = np.zeros((N, 100), bool)
        for t in range(horizon):
            seen[np.arange(N), st[:, 0] * 10 + st[:, 1]] = True
            st, _ = O.darkroom_transit(st, acts[:, e, t], goals, perm=perms)
        distinct[:, e] = seen.sum(1)
    assert np.array_equal(on["forwards"], distinct)
    assert on["forwards"].sum() < off["forwards"].sum()


def test_prefill_equals_positionwise_window():
    """The MFMA prefill (4/8/16 waves: windows of 128/256/512 tokens) and the position-by-position K/V path give the
    same logits (out_mode 0 and 1) on random contexts of every model; both within the bar
    of the reference's recorded logits where fixtures exist."""
    import dpt_hip
    rs = np.random.RandomState(21)
    for name in ("bandit5", "darkroom", "linear20"):
        g, m, _ = model_from_golden(name)
        H, sd, A, L, E = (int(x) for x in g["cfg"])
        assert m.prefill_max_window() == 512
        for N, C in ((3, 0), (37, 5), (64, 100), (17, 127), (9, 128), (20, 255), (5, 300), (6, 500)):
            if C + 1 > 4 * (1 + H):
                continue
            q = rs.randn(N, sd).astype(np.float32)
            cs, cn = rs.randn(N, C, sd).astype(np.float32), rs.randn(N, C, sd).astype(np.float32)
            ca = np.eye(A, dtype=np.float32)[rs.randint(0, A, (N, C))]
            cr = rs.randn(N, C).astype(np.float32)
            outs = []
            try:
                for on in (True, False):
                    dpt_hip.set_prefill(on)
                    for mode in ((0, 1) if C else (0,)):
                        outs.append(m.forward_window(q, cs, ca, cn, cr, out_mode=mode).cpu().numpy())
            finally:
                dpt_hip.set_prefill(True)
            half = len(outs) // 2
            for a, b in zip(outs[:half], outs[half:]):
                assert_logits(a, b)


def test_rollout_bernoulli_philox_vs_oracle():
    """Fused rollout with Bernoulli rewards (r = u < mean, envs/gpu_bandit_env.py:58-61): Philox
    draws through the kernel equal the oracle fed the same uniforms."""
    d = dh()
    _, m, W = model_from_golden("bandit5")
    rs = np.random.RandomState(8)
    N, H, seed = 20, 24, 4242
    means = rs.beta(1, 1, (N, 5))
    out = m.rollout_bandit(means, H, 0.0, True, bandit_type=d.BANDIT_BERNOULLI, seed=seed, want_logits=True)
    u = np.stack([philox_np.uniform(seed, h, np.arange(N), d.STREAM_SELECT) for h in range(H)])
    gu = np.stack([d.draw(0, seed, h, 0, N, d.STREAM_REWARD).cpu().numpy() for h in range(H)])
    ref = O.bandit_online_rollout(W, means, H, 0.0, u, gu, True, bernoulli=True)
    margin = O.boundary_margin(O.softmax_f32(ref["logits"]), u)
    k = H if not (margin < 1e-5).any() else int(np.argmax((margin < 1e-5).any(-1)))
    assert_logits(out["logits"].cpu().numpy()[:k + 1], ref["logits"][:k + 1])
    if k == H:
        assert np.array_equal(out["actions"].cpu().numpy(), ref["actions"])
        assert np.array_equal(out["rewards"].cpu().numpy(), ref["rewards"])
        assert set(np.unique(out["rewards"].cpu().numpy())) <= {0.0, 1.0}


def sampled_tasks(N, tile=8, n_random=48, seed=0):
    """>= 64 tasks of an N-task launch: every slot of the first two tiles (the two workgroups the
    dispatcher puts side by side), the last (possibly partial) tile, and random ones."""
    rs = np.random.RandomState(seed)
    last = (N - 1) // tile * tile
    t = np.concatenate([np.arange(min(N, 2 * tile)), np.arange(last, N), rs.choice(N, n_random, replace=False)])
    return np.unique(t)


def first_tie(margin, bar=1e-5):
    """First step whose uniform lies within ``bar`` of a cdf edge (len(margin) if none)."""
    tie = np.nonzero(margin < bar)[0]
    return int(tie[0]) if tie.size else len(margin)


def compared_steps(acts, ref_acts, margin, bar=1e-5):
    """Per task, the number of leading steps whose trajectory equals the oracle's: the first step
    whose action differs, or all steps.  A differing action is legitimate only at a near-tie draw (a
    uniform within ``bar`` of one of the oracle's cdf edges, where fp32 rounding of the logits may
    decide); anywhere else it fails.  Steps up to and including that one were computed on identical
    windows, so their logits are comparable.  acts, ref_acts: (tasks, steps); margin: (steps, tasks)."""
    steps = acts.shape[1]
    diff = acts != ref_acts
    n = np.where(diff.any(1), diff.argmax(1), steps)
    j = np.nonzero(n < steps)[0]
    flip_margin = margin[n[j], j]
    assert (flip_margin < bar).all(), ("action differs away from a near-tie", j[flip_margin >= bar][:8],
                                       n[j][flip_margin >= bar][:8], flip_margin[flip_margin >= bar][:8])
    return n


@pytest.mark.parametrize("A,H,var,N", [(5, 500, 0.3, 4096), (20, 1000, 0.3, 4096), (5, 500, 0.3, 4093)])
def test_rollout_full_config_all_tasks(A, H, var, N):
    """BASELINE configs 2 (5 arms, H=500) and 4 (20 arms, H=1000; one GPU's 4096-task shard) at full
    size, and config 2 with a partial last tile (4093 tasks): EVERY task of the fused rollout agrees
    with the float64 C oracle (pinned to the reference's rollouts by
    test_c_bandit_oracle_matches_reference; K/V-cache form, bit-identical to its re-forward form)
    fed the same Philox draws -- logits within 1e-5 at every compared step and actions / arm values
    exactly, each task up to its first differing action, which must fall on a near-tie draw (a
    uniform within 1e-5 of a cdf edge, where numpy's own expf decides).  The fraction of task-steps
    compared is printed and must be >= 0.9 (reference: eval_bandit.py:56-103 /
    ctrl_bandit.py:422-444)."""
    import bench
    import dpt_hip
    from oracle import c_oracle
    dh()
    seed, L = 31337, 4
    sd, _ = bench.synthetic_state_dict(L, 1, A, H)
    m = dpt_hip.DeviceModel(sd, L, 1, A, 4 * (1 + H))
    if A == 5:
        means = np.random.RandomState(1).uniform(0, 1, (N, A))
    else:  # collect_data.py:230-231 arms, theta ~ N(0,1)/sqrt(d)
        arms = np.random.RandomState(1234).normal(size=(A, 2)) / np.sqrt(2)
        means = np.random.RandomState(2).normal(0, 1, (N, 2)) / np.sqrt(2) @ arms.T
    out = m.rollout_bandit(means, H, var, True, seed=seed, want_logits=True)
    acts = out["actions"].cpu().numpy()
    av = out["arm_value"].cpu().numpy()
    lg = out["logits"].cpu().numpy()
    del out
    torch.cuda.empty_cache()
    assert np.array_equal(av, means[np.arange(N)[:, None], acts])
    tasks = np.arange(N)
    u = np.stack([philox_np.uniform(seed, h, tasks, dpt_hip.STREAM_SELECT) for h in range(H)])
    g = np.stack([philox_np.normal(seed, h, tasks, dpt_hip.STREAM_REWARD) for h in range(H)])
    blob = dpt_hip.pack_weights(sd, L).numpy()
    ref = c_oracle.bandit_rollout_f64(blob, L, A, 4 * (1 + H), means, H, var, u, g, True, False,
                                      bench.host_cpus()[0], want_logits=True)
    n_cmp = compared_steps(acts, ref["actions"], ref["margin"])  # a differing action only at a near-tie
    step = np.arange(H)[:, None]
    # logits: every step up to and including each task's first differing action
    sel = step <= np.minimum(n_cmp, H - 1)[None, :]
    got, want = lg[sel], ref["logits"][sel]
    bad = np.abs(got - want) > 1e-5 * np.maximum(1, np.abs(want))
    assert not bad.any(), (int(bad.sum()), float(np.abs(got - want).max()))
    okmask = (step < n_cmp[None, :]).T  # (N, H)
    assert np.array_equal(av[okmask], ref["arm_value"][okmask])
    full = float((n_cmp == H).mean())
    print(f"\nA={A} H={H} N={N}: {full:.4f} of tasks identical over all {H} steps, "
          f"{okmask.mean():.5f} of all task-steps compared exactly")
    assert okmask.mean() >= 0.9


def check_darkroom_tasks(out, tasks, ref, Heps, horizon, min_frac=0.9, label=""):
    """Device rollout rows ``tasks`` against the C oracle's rows (same order), every task: actions
    exactly up to the first step whose action differs (which must be a near-tie draw,
    compared_steps), logits within 1e-5 at every step up to and including it, and the returns of
    every episode that ends before it.  The fraction of task-steps compared is printed and must be
    >= ``min_frac``; returns it."""
    steps = Heps * horizon
    lg = out["logits"].cpu().numpy()[:, tasks]
    acts = out["actions"].cpu().numpy()[tasks]
    rets = out["returns"].cpu().numpy()[tasks]
    n = compared_steps(acts, ref["actions"], ref["margin"])
    for j in range(len(tasks)):
        k = min(n[j] + 1, steps)
        assert_logits(lg[:k, j], ref["logits"][:k, j])
        assert np.array_equal(rets[j, :n[j] // horizon], ref["returns"][j, :n[j] // horizon]), tasks[j]
    frac = float(n.sum()) / (len(tasks) * steps)
    print(f"\n{label}: {len(tasks)} tasks, {(n == steps).mean():.4f} of them identical over all {steps} steps, "
          f"{frac:.5f} of task-steps compared exactly")
    assert frac >= min_frac, frac
    return frac


def darkroom_config(N_total, seed=0):
    """SURVEY.md 8(d) C3 / C5 task set: the 100 grid cells in collect_data.py:408-409's
    RandomState(0) shuffle order, cycled over the global task ids."""
    goals = np.array([(j, i) for j in range(10) for i in range(10)])
    np.random.RandomState(0).shuffle(goals)
    return goals[np.arange(N_total) % 100]


def test_rollout_darkroom_full_config3_sampled_tasks():
    """BASELINE config 3 at full size (4096 tasks, Heps=40, horizon=100, goals in collect_data.py's
    shuffled order, logits memo on): 1024+ tasks (the first and last 16 and 1024 random ones) agree
    with the float64 C oracle fed the same Philox draws -- logits within 1e-5, actions and
    per-episode returns exactly, each task up to a flip at a near-tie draw; >= 0.9 of the task-steps
    compared (reference: evals/eval_darkroom.py:53-82)."""
    import bench
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    N, Heps, horizon, seed, ctr, L = 4096, 40, 100, 99, 3, 4
    sd, _ = bench.synthetic_state_dict(L, 2, 5, horizon)
    m = dpt_hip.DeviceModel(sd, L, 2, 5, 4 * (1 + horizon))
    goals = darkroom_config(N)
    out = m.rollout_darkroom(goals, Heps, horizon, 1, seed=seed, counter=ctr, want_actions=True, want_logits=True)
    rs = np.random.RandomState(0)
    tasks = np.unique(np.concatenate([np.arange(16), np.arange(N - 16, N), rs.choice(N, 1024, replace=False)]))
    steps = Heps * horizon
    u = np.stack([philox_np.uniform(seed, ctr + k, tasks, d.STREAM_SELECT) for k in range(steps)])
    ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(sd, L).numpy(), L, 4 * (1 + horizon), goals[tasks], Heps,
                                    horizon, 1, u, True, threads=bench.host_cpus()[0], want_logits=True)
    assert len(tasks) >= 1024
    check_darkroom_tasks(out, tasks, ref, Heps, horizon, label="C3")


@pytest.mark.parametrize("first_task", [0, 57344])
def test_rollout_darkroom_config5_shard(first_task):
    """BASELINE config 5 (DarkRoom, 65,536 tasks over 8 GPUs): one GPU's 8,192-task shard, the first
    and the last rank's, as bench.py runs it (goals of the global ids, Philox keyed by the global
    task id, C3 weights, 40 episodes, memo on): 256+ tasks over both halves of the shard agree
    with the float64 C oracle fed the same draws; >= 0.9 of the task-steps compared."""
    import bench
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    N, Heps, horizon, seed, L = 8192, 40, 100, 1234, 4
    sd, _ = bench.synthetic_state_dict(L, 2, 5, horizon)
    m = dpt_hip.DeviceModel(sd, L, 2, 5, 4 * (1 + horizon))
    goals = darkroom_config(65536)[first_task:first_task + N]
    out = m.rollout_darkroom(goals, Heps, horizon, 1, seed=seed, first_task=first_task, want_actions=True,
                             want_logits=True)
    rs = np.random.RandomState(first_task)
    tasks = np.unique(np.concatenate([[0, 1, 4095, 4096, 8191], rs.choice(4096, 128, replace=False),
                                      4096 + rs.choice(4096, 128, replace=False)]))
    steps = Heps * horizon
    u = np.stack([philox_np.uniform(seed, k, first_task + tasks, d.STREAM_SELECT) for k in range(steps)])
    ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(sd, L).numpy(), L, 4 * (1 + horizon), goals[tasks], Heps,
                                    horizon, 1, u, True, threads=bench.host_cpus()[0], want_logits=True)
    assert len(tasks) >= 256
    check_darkroom_tasks(out, tasks, ref, Heps, horizon, label=f"C5 shard at {first_task}")


def test_empty_batches():
    """No tasks or no steps: empty outputs of the right shapes, no launch (the ABI rejects N=0)."""
    _, m, _ = model_from_golden("bandit5")
    o = m.rollout_bandit(np.zeros((0, 5)), 10, 0.3, True, want_logits=True)
    assert o["actions"].shape == (0, 10) and o["logits"].shape == (10, 0, 5)
    o = m.rollout_bandit(np.random.RandomState(0).uniform(0, 1, (4, 5)), 0, 0.3, True)
    assert o["arm_value"].shape == (4, 0)
    assert m.forward_window(np.zeros((0, 1), np.float32)).shape == (0, 5)
    _, md, _ = model_from_golden("darkroom")
    o = md.rollout_darkroom(np.zeros((0, 2), np.int64), 3, 10, 1, want_forwards=True)
    assert o["returns"].shape == (0, 3) and o["forwards"].shape == (0, 3)


@pytest.mark.parametrize("N,H", [(1000, 500), (4096, 1000), (3, 7)])
def test_regret_moments_match_scipy(N, H):
    """dpt_regret_moments (the eval's regret mean / SEM, evals/eval_bandit.py:169-178) against
    numpy + scipy.stats.sem on the same curves, through distributed.regret_stats_allreduce's
    single-process device path; deterministic run to run."""
    import scipy.stats
    import torch
    from dpt_hip.distributed import regret_stats_allreduce
    rs = np.random.RandomState(N + H)
    means = rs.uniform(0, 1, (N, 5))
    av = means[np.arange(N)[:, None], rs.randint(0, 5, (N, H))] + 3.0  # offset: mean >> spread
    opt = means.max(1) + 3.0
    st = regret_stats_allreduce(torch.from_numpy(opt[:, None]).cuda(), torch.from_numpy(av).cuda(), N)
    st2 = regret_stats_allreduce(torch.from_numpy(opt[:, None]).cuda(), torch.from_numpy(av).cuda(), N)
    for k in st:
        assert torch.equal(st[k], st2[k])
    diff = opt[:, None] - av
    cr = np.cumsum(diff, 1)
    ref = dict(subopt_mean=diff.mean(0), subopt_sem=scipy.stats.sem(diff, 0),
               regret_mean=cr.mean(0), regret_sem=scipy.stats.sem(cr, 0))
    for k, v in ref.items():
        np.testing.assert_allclose(st[k].cpu().numpy(), v, rtol=1e-10, atol=1e-12)


def test_rollout_darkroom_workspace_matches_lds_path():
    """With the per-episode workspace (context tokens' layer-0 inputs, queries and attention
    partials kept instead of recomputed each step) the rollout keeps the values as split tiles
    and runs both attention products on the split bf16 matrix cores; without it the values stay
    fp32 and P V runs on 16x16x4_f32.  Same forward up to fp32 rounding: per task the logits agree
    within the 1e-5 bar up to the first step whose sampled action differs (a uniform within
    rounding of a cdf edge), and such divergences are rare."""
    import dpt_hip
    _, m, _ = model_from_golden("darkroom")
    rs = np.random.RandomState(23)
    N, steps = 300, 400
    goals = rs.randint(0, 10, (N, 2))
    outs = []
    try:
        for on in (False, True):
            dpt_hip.set_darkroom_workspace(on)
            o = m.rollout_darkroom(goals, 4, 100, 1, seed=4, want_actions=True, want_logits=True)
            outs.append({k: o[k].cpu().numpy() for k in ("actions", "logits", "returns")})
    finally:
        dpt_hip.set_darkroom_workspace(True)
    diff = outs[0]["actions"] != outs[1]["actions"]
    first = np.where(diff.any(1), diff.argmax(1), steps)  # first differing step per task
    assert (first < steps).mean() <= 0.01
    same = first == steps
    assert np.array_equal(outs[0]["returns"][same], outs[1]["returns"][same])
    for t in range(N):
        f = min(first[t] + 1, steps)  # logits of steps <= first[t] were computed on identical windows
        assert_logits(outs[1]["logits"][:f, t], outs[0]["logits"][:f, t])


@pytest.mark.parametrize("factor", [1.0 / 64, 4.0, 8.0])
def test_prefill_fp16_split_scales_follow_the_weights(factor):
    """The window forwards run every product as fp16 two-part split products whose power-of-two
    scales come from static bounds on the weights (dpt_abi.hip fwd_scales).  With the block
    weights scaled by 1/64, 4 or 8 (and the LayerNorm gains by 3 for the large factors, so scores
    and activations grow too) nothing overflows fp16 and small values keep their precision: against
    the float64 oracle the MFMA prefill is as accurate as the fp32 position-by-position path (within
    the logit bar, or within twice the fp32 path's own error where large scores make fp32 itself
    miss it: factor 8 gives 5.0e-5 vs 3.8e-5, scripts/scale_stress.py)."""
    import dpt_hip
    g = golden("forward_darkroom.npz")
    H, sd, A, L, E = (int(x) for x in g["cfg"])
    w = {}
    for k, v in g.items():
        if not k.startswith("w/"):
            continue
        t = v.astype(np.float32).copy()
        if any(s in k for s in ("c_fc.weight", "c_proj.weight", "c_attn.weight")):
            t *= factor
        if factor > 1 and ("ln_1.weight" in k or "ln_2.weight" in k):
            t *= 3.0
        w[k[2:]] = t
    m = dpt_hip.DeviceModel({k: torch.from_numpy(v) for k, v in w.items()}, L, sd, A, 4 * (1 + H))
    W = O.split_weights(w, L)
    rs = np.random.RandomState(31)
    for N, C in ((32, 100), (6, 300)):
        q = rs.randn(N, sd).astype(np.float32)
        cs, cn = rs.randn(N, C, sd).astype(np.float32), rs.randn(N, C, sd).astype(np.float32)
        ca = np.eye(A, dtype=np.float32)[rs.randint(0, A, (N, C))]
        cr = rs.randn(N, C).astype(np.float32)
        ref = O.transformer_forward(W, q, cs, ca, cn, cr, test=True)
        err = {}
        try:
            for on in (True, False):
                dpt_hip.set_prefill(on)
                lg = m.forward_window(q, cs, ca, cn, cr).cpu().numpy().astype(np.float64)
                assert np.isfinite(lg).all()
                err[on] = float((np.abs(lg - ref) / np.maximum(1.0, np.abs(ref))).max())
        finally:
            dpt_hip.set_prefill(True)
        assert err[True] <= max(LOGIT_TOL, 2.0 * err[False]), err


def test_rollout_darkroom_dim12_workspace_without_state_table():
    """dim = 12 (144 grid cells > the 128-row state table): with the workspace but no per-state
    query table the kernel re-embeds block 0 and takes the query token's key / value through
    its own branch.  Workspace on vs off agree within the logit bar up to the first differing
    sampled action, and sampled tasks agree with the float64 C oracle fed the same draws."""
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    g, m, _ = model_from_golden("darkroom")
    N, Heps, horizon, R, dim, seed = 256, 5, 40, 2, 12, 21
    goals = np.random.RandomState(12).randint(0, dim, (N, 2))
    outs = []
    try:
        for on in (False, True):
            dpt_hip.set_darkroom_workspace(on)
            o = m.rollout_darkroom(goals, Heps, horizon, R, dim=dim, seed=seed, want_actions=True, want_logits=True)
            outs.append(o)
    finally:
        dpt_hip.set_darkroom_workspace(True)
    steps = Heps * horizon
    a0, a1 = (o["actions"].cpu().numpy() for o in outs)
    diff = a0 != a1
    first = np.where(diff.any(1), diff.argmax(1), steps)
    assert (first < steps).mean() <= 0.02
    l0, l1 = (o["logits"].cpu().numpy() for o in outs)
    for t in range(N):
        f = min(first[t] + 1, steps)
        assert_logits(l1[:f, t], l0[:f, t])
    tasks = np.arange(0, N, 17)
    u = np.stack([philox_np.uniform(seed, k, tasks, d.STREAM_SELECT) for k in range(steps)])
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")}
    ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(w, 4).numpy(), 4, 404, goals[tasks], Heps, horizon, R, u,
                                    True, dim=dim, threads=16, want_logits=True)
    check_darkroom_tasks(outs[1], tasks, ref, Heps, horizon, label="dim 12 workspace")


_NOWS_REF = {}


@pytest.mark.parametrize("memo", [False, True])
@pytest.mark.parametrize("R", [1, 2])
@pytest.mark.parametrize("dim", [11, 12])
def test_rollout_darkroom_workspace_free_vs_oracle(dim, R, memo):
    """The workspace-free kernels (rollout_darkroom_kernel<false, 4|8, false>, step specialised on
    the wave's block count) on grids over 10 x 10: dim 11 with the workspace switched off and dim 12,
    which takes them by default (144 cells exceed the per-state table), at windows 101 (4 waves;
    episodes of 1, 101, 101 tokens) and 201 (8 waves; 1, 101, 201, 201), memo off and on (dim 12
    has no memo: more cells than memo rows).  This is where a 3e-3 logit error was once observed
    (workspace-free kernels).  EVERY task of a 256-task batch agrees with the float64 C
    oracle fed the same Philox draws: logits within 1e-5, actions and per-episode returns exactly,
    each task up to a flip at a near-tie draw; >= 0.9 of the task-steps compared (reference:
    evals/eval_darkroom.py:20-84, ctrls/ctrl_darkroom.py:23-66)."""
    import bench
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    L, horizon, N, seed = 4, 100, 256, 4242 + dim
    Heps = R + 2
    sd, _ = bench.synthetic_state_dict(L, 2, 5, R * horizon)
    m = dpt_hip.DeviceModel(sd, L, 2, 5, 4 * (1 + R * horizon))
    goals = np.random.RandomState(dim).randint(0, dim, (N, 2))
    try:
        dpt_hip.set_darkroom_workspace(False)
        dpt_hip.set_darkroom_memo(memo)
        out = m.rollout_darkroom(goals, Heps, horizon, R, dim=dim, seed=seed, want_actions=True, want_logits=True,
                                 want_forwards=True)
    finally:
        dpt_hip.set_darkroom_workspace(True)
        dpt_hip.set_darkroom_memo(True)
    fw = out["forwards"].cpu().numpy()
    if memo and dim * dim <= 128:
        assert fw.sum() < N * Heps * horizon
    else:
        assert (fw == horizon).all()
    steps = Heps * horizon
    if (dim, R) not in _NOWS_REF:  # the oracle does not depend on the memo switch
        tasks = np.arange(N)
        u = np.stack([philox_np.uniform(seed, k, tasks, d.STREAM_SELECT) for k in range(steps)])
        _NOWS_REF[dim, R] = c_oracle.darkroom_rollout(dpt_hip.pack_weights(sd, L).numpy(), L, 4 * (1 + R * horizon),
                                                      goals, Heps, horizon, R, u, True, dim=dim,
                                                      threads=bench.host_cpus()[0], want_logits=True)
    check_darkroom_tasks(out, np.arange(N), _NOWS_REF[dim, R], Heps, horizon,
                         label=f"workspace-free dim {dim} window {1 + R * horizon} memo {memo}")


@pytest.mark.parametrize("Heps,horizon,R,dim", [(4, 100, 3, 10), (2, 511, 1, 10), (2, 300, 1, 12)])
def test_rollout_darkroom_windows_over_256(Heps, horizon, R, dim):
    """Windows of 257..512 tokens run the 16-wave kernel (one task per CU, keys and values of the
    whole window in LDS): window 301 (the reference's H = 300 with horizon 100, episodes of 1, 101,
    201 and 301 tokens) and 512 (the largest).  The logits memo is bit-identical to one forward per
    step, and sampled tasks agree with the float64 C oracle fed the same Philox draws (logits within
    1e-5, actions and returns exactly up to each task's first near-tie draw).  Without the
    workspace these windows are rejected (NotImplementedError: use the per-step path).  dim = 12
    (144 states) runs without the per-state query table and the memo (both need <= 128 states)."""
    import bench
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    L, npos = 4, 512
    sd, _ = bench.synthetic_state_dict(L, 2, 5, npos // 4 - 1)
    m = dpt_hip.DeviceModel(sd, L, 2, 5, npos)
    N, seed = 48, 5
    goals = darkroom_config(N)
    steps = Heps * horizon
    outs = {}
    try:
        for memo in (True, False):
            dpt_hip.set_darkroom_memo(memo)
            o = m.rollout_darkroom(goals, Heps, horizon, R, dim=dim, seed=seed, want_actions=True, want_logits=True,
                                   want_forwards=True)
            outs[memo] = {k: o[k].cpu().numpy() for k in ("actions", "logits", "returns", "forwards")}
        dpt_hip.set_darkroom_workspace(False)
        with pytest.raises(NotImplementedError):
            m.rollout_darkroom(goals[:2], 1, horizon, R)
    finally:
        dpt_hip.set_darkroom_workspace(True)
        dpt_hip.set_darkroom_memo(True)
    on, off = outs[True], outs[False]
    for k in ("actions", "logits", "returns"):
        assert np.array_equal(on[k], off[k]), k
    assert (off["forwards"] == horizon).all()
    assert on["forwards"].sum() < off["forwards"].sum() if dim * dim <= 128 else (on["forwards"] == horizon).all()
    tasks = np.arange(0, N, 3)
    u = np.stack([philox_np.uniform(seed, k, tasks, d.STREAM_SELECT) for k in range(steps)])
    ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(sd, L).numpy(), L, npos, goals[tasks], Heps, horizon, R, u,
                                    True, dim=dim, threads=16, want_logits=True)
    res = {k: torch.from_numpy(on[k]) for k in ("logits", "actions", "returns")}
    check_darkroom_tasks(res, tasks, ref, Heps, horizon, label=f"window {1 + R * horizon}")


@pytest.mark.parametrize("Heps,horizon,R", [(4, 100, 2), (3, 85, 3)])
def test_rollout_darkroom_long_windows(Heps, horizon, R):
    """Windows of 129..256 tokens run the 8-wave kernel (two 16-token blocks per wave): window 201
    (the reference's H = 200 with horizon 100) and 256 (the largest).  Sampled tasks agree with the
    float64 C oracle fed the same Philox draws (logits within 1e-5, actions and returns exactly up
    to each task's first near-tie draw); the logits memo is bit-identical to one forward per step;
    the workspace and LDS-only variants agree within the logit bar up to the first differing
    sampled action."""
    import dpt_hip
    from oracle import c_oracle
    d = dh()
    g, m, _ = model_from_golden("darkroom")
    N, seed = 192, 77
    goals = darkroom_config(N)
    steps = Heps * horizon
    outs = {}
    try:
        for ws, memo in ((True, True), (True, False), (False, True)):
            dpt_hip.set_darkroom_workspace(ws)
            dpt_hip.set_darkroom_memo(memo)
            o = m.rollout_darkroom(goals, Heps, horizon, R, seed=seed, want_actions=True, want_logits=True,
                                   want_forwards=True)
            outs[ws, memo] = {k: o[k].cpu().numpy() for k in ("actions", "logits", "returns", "forwards")}
    finally:
        dpt_hip.set_darkroom_workspace(True)
        dpt_hip.set_darkroom_memo(True)
    on, off = outs[True, True], outs[True, False]
    for k in ("actions", "logits", "returns"):
        assert np.array_equal(on[k], off[k]), k
    assert (off["forwards"] == horizon).all() and on["forwards"].sum() < off["forwards"].sum()
    lds = outs[False, True]
    diff = lds["actions"] != on["actions"]
    first = np.where(diff.any(1), diff.argmax(1), steps)
    assert (first < steps).mean() <= 0.02
    for t in range(N):
        f = min(first[t] + 1, steps)
        assert_logits(lds["logits"][:f, t], on["logits"][:f, t])
    tasks = np.arange(0, N, 3)
    u = np.stack([philox_np.uniform(seed, k, tasks, d.STREAM_SELECT) for k in range(steps)])
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")}
    ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(w, 4).numpy(), 4, 404, goals[tasks], Heps, horizon, R, u,
                                    True, threads=16, want_logits=True)
    res = {"logits": torch.from_numpy(on["logits"]), "actions": torch.from_numpy(on["actions"]),
           "returns": torch.from_numpy(on["returns"])}
    assert len(tasks) >= 64
    check_darkroom_tasks(res, tasks, ref, Heps, horizon, label=f"window {1 + R * horizon}")


def test_rollout_bandit_stream_base_bit31():
    """Regression for the round-4 GPU fault: rollout_bandit_kernel builds a buffer descriptor per
    task stream from its base address, which once went through readfirstlane(int) and was
    sign-extended when bit 31 of the base's low word was set (an illegal address).  The K/V
    workspace is placed inside a larger allocation so that every stream base of the launch has
    bit 31 of its low word set; the rollout must equal the one on an ordinary allocation bit for
    bit.  Run once per suite; it is not a fault reproducer to loop on."""
    _, m, _ = model_from_golden("bandit5")
    N, H, seed = 64, 40, 77
    means = np.random.RandomState(5).uniform(0, 1, (N, 5))
    ref = m.rollout_bandit(means, H, 0.3, True, seed=seed, want_logits=True)
    need = m.kv_numel(N, H)
    assert need * 4 < (1 << 30)  # the whole workspace stays inside one 2 GiB half of the low word
    big = torch.empty((1 << 30) + need + 1024, dtype=torch.float32, device="cuda")  # 4 GiB + workspace
    off = ((0x80000000 + 0x400) - (big.data_ptr() & 0xFFFFFFFF)) % (1 << 32)
    assert off % 4 == 0
    kv = big[off // 4:off // 4 + need]
    lo, hi = kv.data_ptr() & 0xFFFFFFFF, (kv.data_ptr() + 4 * need - 1) & 0xFFFFFFFF
    assert lo >> 31 == 1 and hi >> 31 == 1 and hi > lo
    out = m.rollout_bandit(means, H, 0.3, True, seed=seed, want_logits=True, kvcache=kv)
    torch.cuda.synchronize()
    for k in ("actions", "rewards", "arm_value", "logits"):
        assert torch.equal(out[k], ref[k]), k
    del big, kv, out
    torch.cuda.empty_cache()
