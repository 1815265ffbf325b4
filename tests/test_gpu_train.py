"""The training path: dpt_train_forward / dpt_train_backward through the
drop-in Transformer, against gradients recorded from the reference's train.py loss
(tests/golden/train_grads.npz, float64) and the float64 torch oracle (oracle/dpt_oracle_torch.py).

Bars: preds within 1e-5 * max(1, |x|) (the logit bar); every parameter's gradient within
GRAD_TOL of the largest entry of its float64 gradient (the reference's own fp32 run is at
3.5e-7 of it; the HIP kernels sum over the batch * window rows in a different order)."""
import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu

GRAD_TOL = 2e-5
KEYS = ("query_states", "context_states", "context_actions", "context_next_states", "context_rewards")


def model_from_fixture(name, n_embd=None):
    from models.net import Transformer
    fw = golden(f"forward_{name}.npz")
    H, sd, A, L, E = (int(x) for x in fw["cfg"])
    m = Transformer(dict(horizon=H, state_dim=sd, action_dim=A, n_layer=L, n_embd=E, n_head=4, dropout=0.0,
                         test=False))
    state = {k[2:]: torch.from_numpy(v) for k, v in fw.items() if k.startswith("w/")}
    state["transformer.wte.weight"] = m.transformer.wte.weight.detach().clone()
    m.load_state_dict(state)
    return fw, m.cuda()


def batch_from(g, name):
    b = {k: torch.from_numpy(g[f"{name}/{k}"]).float().cuda() for k in KEYS}
    b["zeros"] = torch.from_numpy(g[f"{name}/zeros"]).float().cuda()
    return b, torch.from_numpy(g[f"{name}/optimal_actions"]).float().cuda()


def rel_err(got, ref):
    return float(np.abs(np.asarray(got, np.float64) - ref).max() / max(1e-30, np.abs(ref).max()))


@pytest.mark.parametrize("name", ["darkroom", "bandit5"])
def test_train_step_gradients_match_reference(name):
    """The reference's training step (train.py:296-310) on our Transformer: forward in training
    mode, CrossEntropyLoss(sum) over preds[:, 1:], loss.backward() -> every parameter's .grad
    from the HIP backward; loss, preds and gradients against the reference's float64 values."""
    g = golden("train_grads.npz")
    fw, m = model_from_fixture(name)
    A = int(fw["cfg"][2])
    batch, opt = batch_from(g, name)
    m.train()
    pred = m(batch)
    true = opt.unsqueeze(1).repeat(1, pred.shape[1], 1).reshape(-1, A)
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, A), true)
    m.zero_grad()
    loss.backward()
    ref_loss = float(g[f"{name}/f64/loss"])
    assert abs(loss.item() - ref_loss) <= 1e-5 * abs(ref_loss)
    ref = g[f"{name}/f64/preds"]
    assert (np.abs(pred.detach().cpu().numpy() - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all()
    worst = 0.0
    for k, p in m.named_parameters():
        if k.endswith("wte.weight"):
            assert p.grad is None
            continue
        ref = g[f"{name}/f64/grad/{k}"]
        got = p.grad.detach().cpu().numpy()
        if k.endswith("wpe.weight"):
            assert not got[ref.shape[0]:].any()
            got = got[:ref.shape[0]]
        e = rel_err(got, ref)
        worst = max(worst, e)
        assert e <= GRAD_TOL, (k, e)
    print(f"{name}: worst gradient error {worst:.2e} of max |g|")


def test_adamw_steps_track_the_float64_oracle():
    """Three AdamW steps (train.py:254, lr 1e-3, weight decay 1e-4) on the HIP gradients track the
    same steps taken on the float64 oracle's gradients: the losses agree within 1e-5 at every step
    and >= 99.5 % of the parameter entries within 1e-5 (Adam divides each gradient by its own
    running magnitude, so an entry whose gradient is ~0 in float64 can take a different-sign step
    of up to 2 lr from fp32 rounding; every entry stays within that bound)."""
    from oracle import dpt_oracle_torch as OT
    g = golden("train_grads.npz")
    fw, m = model_from_fixture("darkroom")
    L, sd, A = int(fw["cfg"][3]), int(fw["cfg"][1]), int(fw["cfg"][2])
    batch, opt = batch_from(g, "darkroom")
    P = OT.state_dict_params({k[2:]: v for k, v in fw.items() if k.startswith("w/")}, L)
    names = list(P)
    lr, steps = 1e-3, 3
    opt_ref = torch.optim.AdamW([P[k] for k in names], lr=lr, weight_decay=1e-4)
    params = dict(m.named_parameters())
    opt_hip = torch.optim.AdamW([params[k] for k in names], lr=lr, weight_decay=1e-4)
    hb = {k: g[f"darkroom/{k}"] for k in KEYS}
    hb["optimal_actions"] = g["darkroom/optimal_actions"]
    m.train()
    for _ in range(steps):
        pred = m(batch)
        true = opt.unsqueeze(1).repeat(1, pred.shape[1], 1).reshape(-1, A)
        loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, A), true)
        opt_hip.zero_grad()
        loss.backward()
        opt_hip.step()
        opt_ref.zero_grad()
        ref_loss = OT.train_loss(P, hb, L, sd, A)[0]
        ref_loss.backward()
        opt_ref.step()
        assert abs(loss.item() - ref_loss.item()) <= 1e-5 * abs(ref_loss.item())
    diffs = np.concatenate([np.abs(params[k].detach().cpu().numpy() - P[k].detach().numpy()).ravel()
                            for k in names])
    assert (diffs <= 1e-5).mean() >= 0.995, (diffs <= 1e-5).mean()
    assert diffs.max() <= 2 * lr * steps + 1e-5


@pytest.mark.parametrize("name,B,C", [("darkroom", 16, 100), ("bandit5", 4, 500)])
def test_train_gradients_full_windows_vs_oracle(name, B, C):
    """Full-length windows (DarkRoom 1 + 100 tokens, bandit 1 + 500: the configs' horizons)
    against the float64 oracle on random contexts."""
    from oracle import dpt_oracle_torch as OT
    fw, m = model_from_fixture(name)
    H, sd, A, L, _ = (int(x) for x in fw["cfg"])
    rs = np.random.RandomState(B + C)
    hb = {"query_states": rs.randint(0, 10, (B, sd)).astype(np.float64),
          "context_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_actions": np.eye(A)[rs.randint(0, A, (B, C))],
          "context_next_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_rewards": rs.normal(0.5, 0.5, (B, C, 1)), "optimal_actions": np.eye(A)[rs.randint(0, A, B)]}
    loss_ref, preds_ref, grads_ref = OT.grads({k[2:]: v for k, v in fw.items() if k.startswith("w/")}, hb, L, sd, A)
    batch = {k: torch.tensor(hb[k], dtype=torch.float32, device="cuda") for k in KEYS}
    batch["zeros"] = torch.zeros((B, sd * sd + A + 1), device="cuda")
    m.train()
    pred = m(batch)
    true = torch.tensor(hb["optimal_actions"], dtype=torch.float32, device="cuda")
    true = true.unsqueeze(1).repeat(1, pred.shape[1], 1).reshape(-1, A)
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, A), true)
    m.zero_grad()
    loss.backward()
    assert abs(loss.item() - loss_ref) <= 1e-5 * abs(loss_ref)
    assert (np.abs(pred.detach().cpu().numpy() - preds_ref) <= 1e-5 * np.maximum(1, np.abs(preds_ref))).all()
    for k, p in m.named_parameters():
        if k.endswith("wte.weight"):
            continue
        e = rel_err(p.grad.detach().cpu().numpy(), grads_ref[k])
        assert e <= 5 * GRAD_TOL, (k, e)


@pytest.mark.parametrize("E,sd,T", [(16, 2, 103), (64, 2, 103), (16, 1, 38), (64, 1, 38)])
def test_train_gradients_other_widths_vs_oracle(E, sd, T):
    """The matrix-core training kernels at widths 16 and 64 (tr_mm_rows / tr_wgrad_mfma /
    tr_attn_*_mfma instantiations other than E = 32): every parameter's gradient against the
    float64 oracle.  Windows with T % 16 != 0 and T % 4 != 0 cover the padded P / dS rows and the
    partial key tiles."""
    from models.net import Transformer
    from oracle import dpt_oracle_torch as OT
    A, L, B, C = 5, 3, 6, T - 1
    torch.manual_seed(E + T)
    m = Transformer(dict(horizon=C, state_dim=sd, action_dim=A, n_layer=L, n_embd=E, n_head=1, dropout=0.0,
                         test=False))
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    w = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    m = m.cuda()
    rs = np.random.RandomState(E * 7 + T)
    hb = {"query_states": rs.randint(0, 10, (B, sd)).astype(np.float64),
          "context_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_actions": np.eye(A)[rs.randint(0, A, (B, C))],
          "context_next_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_rewards": rs.normal(0.5, 0.5, (B, C, 1)), "optimal_actions": np.eye(A)[rs.randint(0, A, B)]}
    loss_ref, preds_ref, grads_ref = OT.grads(w, hb, L, sd, A)
    batch = {k: torch.tensor(hb[k], dtype=torch.float32, device="cuda") for k in KEYS}
    batch["zeros"] = torch.zeros((B, sd * sd + A + 1), device="cuda")
    m.train()
    pred = m(batch)
    true = torch.tensor(hb["optimal_actions"], dtype=torch.float32, device="cuda")
    true = true.unsqueeze(1).repeat(1, pred.shape[1], 1).reshape(-1, A)
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, A), true)
    m.zero_grad()
    loss.backward()
    assert abs(loss.item() - loss_ref) <= 1e-5 * abs(loss_ref)
    assert (np.abs(pred.detach().cpu().numpy() - preds_ref) <= 1e-5 * np.maximum(1, np.abs(preds_ref))).all()
    for k, p in m.named_parameters():
        if k.endswith("wte.weight"):
            continue
        e = rel_err(p.grad.detach().cpu().numpy(), grads_ref[k])
        assert e <= 5 * GRAD_TOL, (k, e)


def test_forward_only_flag_under_autograd_raises():
    """FORWARD_ONLY requested while parameters require grad: the backward names that cause."""
    from dpt_hip import train as tr
    g = golden("train_grads.npz")
    _, m = model_from_fixture("bandit5")
    batch, _ = batch_from(g, "bandit5")
    tok = m._tokens(batch)
    dims = (m.n_layer, m.n_embd, m.state_dim, m.action_dim, m.n_positions, tok.shape[0], tok.shape[1],
            tr.FORWARD_ONLY)
    preds = tr.TransformerFunction.apply(tok, dims, *tr.param_list(m))
    with pytest.raises(RuntimeError, match="FORWARD_ONLY"):
        preds.square().sum().backward()


def test_train_backward_deterministic():
    """Two backward passes of the same batch give bit-identical gradients (fixed-order sums)."""
    g = golden("train_grads.npz")
    _, m = model_from_fixture("bandit5")
    batch, opt = batch_from(g, "bandit5")
    m.train()
    outs = []
    for _ in range(2):
        m.zero_grad()
        m(batch).square().sum().backward()
        outs.append([p.grad.clone() for p in m.parameters() if p.grad is not None])
    assert all(torch.equal(a, b) for a, b in zip(*outs))


@pytest.mark.parametrize("E", [16, 64])
def test_other_widths_forward_and_rollout(E):
    """models/net.py builds GPT2Config(n_embd=self.n_embd) from --embd (common_args.py:31): widths
    other than 32 run the generic kernels.  Forward logits (test=True and test=False) within 1e-5
    of the float64 oracle, and the bandit online loop with such a model runs through the per-step
    device path (cum_means equal to the oracle rollout fed the same draws)."""
    from models.net import Transformer
    from oracle import dpt_oracle as O
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    torch.manual_seed(E)
    m = Transformer(dict(horizon=20, state_dim=1, action_dim=5, n_layer=3, n_embd=E, n_head=1, dropout=0.0,
                         test=True)).cuda().eval()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    W = O.split_weights({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, 3)
    rs = np.random.RandomState(E)
    N, C = 6, 15
    q, cs, cn = np.ones((N, 1)), np.ones((N, C, 1)), np.ones((N, C, 1))
    ca, cr = np.eye(5)[rs.randint(0, 5, (N, C))], rs.normal(0.5, 0.5, (N, C, 1))
    b = {"query_states": torch.tensor(q).float(), "zeros": torch.zeros(N, 7),
         "context_states": torch.tensor(cs).float(), "context_actions": torch.tensor(ca).float(),
         "context_next_states": torch.tensor(cn).float(), "context_rewards": torch.tensor(cr).float()}
    for test in (True, False):
        m.test = test
        got = m(b).detach().cpu().numpy()  # eval mode with grad enabled builds a graph, as the reference's does
        ref = O.transformer_forward(W, q, cs, ca, cn, cr, test=test)
        assert (np.abs(got - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all(), test
    m.test = True
    H, n = 12, 5
    means = rs.uniform(0, 1, (n, 5))
    u, gg = rs.uniform(size=(H, n)), rs.normal(size=(H, n))
    vec = BanditEnvVec([BanditEnv(mu, H, var=0.3) for mu in means])
    ctrl = BanditTransformerController(m, sample=True, batch_size=n)
    cm = eval_bandit.deploy_online_vec(vec, ctrl, H, uniforms=u, noise=gg)
    ref = O.bandit_online_rollout(W, means, H, 0.3, u, gg)
    assert np.array_equal(cm, ref["cum_means"])


@pytest.mark.parametrize("E", [16, 64])
def test_other_widths_darkroom_offline(E):
    """evals/eval_darkroom.py offline (:124-189) with a model of width != 32: the DPT legs run the
    controller's per-step forward (the generic kernels) and match the float64 oracle's episode fed
    the same uniforms (sampled) and greedily."""
    import matplotlib
    matplotlib.use("Agg")
    from models.net import Transformer
    from oracle import dpt_oracle as O
    from evals import eval_darkroom
    torch.manual_seed(E + 1)
    m = Transformer(dict(horizon=10, state_dim=2, action_dim=5, n_layer=2, n_embd=E, n_head=1, dropout=0.0,
                         test=True)).cuda().eval()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.3 * torch.randn_like(p))
    W = O.split_weights({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, 2)
    rs = np.random.RandomState(E)
    n, H = 4, 10
    goals = rs.randint(0, 10, (n, 2))
    trajs = [{"goal": goals[i], "context_states": rs.randint(0, 10, (H, 2)),
              "context_actions": np.eye(5)[rs.randint(0, 5, H)], "context_next_states": rs.randint(0, 10, (H, 2)),
              "context_rewards": rs.randint(0, 2, H)} for i in range(n)]
    u = rs.uniform(size=(H, n))
    res = eval_darkroom.offline(trajs, m, n_eval=n, H=H, dim=10, uniforms=u)
    ctx = tuple(np.stack([t[k] for t in trajs]).astype(np.float64) for k in
                ("context_states", "context_actions", "context_next_states"))
    ctx = ctx + (np.stack([t["context_rewards"] for t in trajs])[..., None].astype(np.float64),)
    assert np.array_equal(res["Opt"], O.darkroom_opt_returns(goals, H))
    assert np.array_equal(res["Learner"], O.darkroom_offline_episode(W, goals, ctx, H, u, sample=True).sum(-1))
    assert np.array_equal(res["Learner (greedy)"],
                          O.darkroom_offline_episode(W, goals, ctx, H, None, sample=False).sum(-1))


@pytest.mark.parametrize("E,memo", [(16, True), (64, True), (16, False)])
def test_other_widths_darkroom_online(E, memo):
    """evals/eval_darkroom.py deploy_online_vec (:20-84) with a model of width != 32: the per-step
    device loop (generic kernels, the per-episode logits memo, device selection and grid step)
    against the float64 oracle's rollout fed the same uniforms: returns and actions exactly, with
    the memo and without it."""
    import dpt_hip
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec
    from evals import eval_darkroom
    from models.net import Transformer
    from oracle import dpt_oracle as O
    torch.manual_seed(E + 7)
    horizon, R, Heps, n = 10, 2, 5, 24
    m = Transformer(dict(horizon=R * horizon, state_dim=2, action_dim=5, n_layer=2, n_embd=E, n_head=1,
                         dropout=0.0, test=True)).cuda().eval()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.3 * torch.randn_like(p))
    W = O.split_weights({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, 2)
    rs = np.random.RandomState(E)
    goals = rs.randint(0, 10, (n, 2))
    u = rs.uniform(size=(Heps, horizon, n))
    ref = O.darkroom_online_rollout(W, goals, Heps, R * horizon, horizon, u)
    vec = DarkroomEnvVec([DarkroomEnv(10, g, horizon) for g in goals])
    ctrl = DarkroomTransformerController(m, batch_size=n, sample=True)
    uf = u.reshape(-1, n)
    ctrl.uniforms = lambda k: uf[k]
    assert eval_darkroom._device_ok(vec, ctrl) and not eval_darkroom._fused_ok(vec, ctrl, R * horizon)
    try:
        dpt_hip.set_darkroom_memo(memo)
        ret = eval_darkroom.deploy_online_vec(vec, ctrl, Heps, R * horizon, horizon)
    finally:
        dpt_hip.set_darkroom_memo(True)
    assert np.array_equal(ret, ref["returns"])


@pytest.mark.parametrize("E,T", [(16, 38), (48, 101), (64, 101), (32, 1)])
def test_forward_last_position_only(E, T):
    """DPT_TRAIN_LAST_ONLY (Transformer.forward in test mode without autograd): the last block runs
    for the last position alone; preds[:, -1] agrees with the full forward-only pass within the logit
    bar at widths on the matrix cores (16, 64), on the row kernels (48), and at T = 1 (the flag is a
    no-op there)."""
    from dpt_hip import train as tr
    m = _width_model(E, 3, max(T, 2), E + T)
    rs = np.random.RandomState(E + T)
    B = 9
    tok = torch.from_numpy(rs.randn(B, T, 2 + 5 + 1).astype(np.float32)).cuda()
    dims = (m.n_layer, m.n_embd, m.state_dim, m.action_dim, m.n_positions, B, T)
    blob = tr.pack_params(tr.param_list(m), torch.device("cuda"))
    full, _ = tr.forward(tr.desc(*dims, flags=tr.FORWARD_ONLY), blob, tok)
    last, _ = tr.forward(tr.desc(*dims, flags=tr.FORWARD_ONLY | tr.LAST_ONLY), blob, tok)
    a, b = last[:, -1].cpu().numpy(), full[:, -1].cpu().numpy()
    assert (np.abs(a - b) <= 1e-5 * np.maximum(1, np.abs(b))).all(), np.abs(a - b).max()
    with pytest.raises(ValueError, match="LAST_ONLY"):
        tr.forward(tr.desc(*dims, flags=tr.LAST_ONLY), blob, tok)


def test_forward_only_workspace_and_second_backward():
    """Without autograd the generic forward runs on the forward-only workspace (DPT_TRAIN_FORWARD_ONLY:
    one layer's activations, no attention probabilities): same preds bit for bit as the training
    forward, a far smaller workspace, and dpt_train_backward refuses that desc.  A second backward
    through one graph (retain_graph=True) raises an explicit error."""
    import dpt_hip
    from dpt_hip import train as tr
    g = golden("train_grads.npz")
    _, m = model_from_fixture("bandit5")
    batch, _ = batch_from(g, "bandit5")
    m.train()
    full = m._forward_generic(batch)
    with torch.no_grad():
        fwd_only = m._forward_generic(batch)
    assert torch.equal(full.detach(), fwd_only)
    tok = m._tokens(batch)
    dims = (m.n_layer, m.n_embd, m.state_dim, m.action_dim, m.n_positions, tok.shape[0], tok.shape[1])
    n_full = tr._numel("dpt_train_workspace_numel", tr.desc(*dims))
    n_inf = tr._numel("dpt_train_workspace_numel", tr.desc(*dims, flags=tr.FORWARD_ONLY))
    assert n_inf * 3 < n_full, (n_inf, n_full)
    d = tr.desc(*dims, flags=tr.FORWARD_ONLY)
    blob = tr.pack_params(tr.param_list(m), dpt_hip.device())
    preds, ws = tr.forward(d, blob, tok)
    assert torch.equal(preds[:, 1:], full.detach())
    with pytest.raises(ValueError, match="forward-only"):
        tr.backward(d, blob, tok, ws, torch.ones_like(preds))
    loss = full.square().sum()
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="retain_graph"):
        loss.backward()


def _dropout_step(m, batch, opt, A, p, seed, grad=True):
    """One train.py:296-310 step of m in training mode with dropout p through
    TransformerFunction with an explicit mask seed -> (loss, preds[:, 1:])."""
    from dpt_hip import train as tr
    tok = m._tokens(batch)
    dims = (m.n_layer, m.n_embd, m.state_dim, m.action_dim, m.n_positions, tok.shape[0], tok.shape[1],
            0 if grad else tr.FORWARD_ONLY, p, seed)
    pred = tr.TransformerFunction.apply(tok, dims, *tr.param_list(m))[:, 1:, :]
    true = opt.unsqueeze(1).repeat(1, pred.shape[1], 1).reshape(-1, A)
    loss = torch.nn.CrossEntropyLoss(reduction="sum")(pred.reshape(-1, A), true)
    if grad:
        m.zero_grad()
        loss.backward()
    return loss, pred


@pytest.mark.parametrize("case", [0, 1])
def test_train_dropout_matches_reference(case):
    """Training-mode dropout (models/net.py:30-32, p = 0.1 and 0.3): loss, preds and every
    gradient against the reference model run with the same masks injected
    (tests/golden/train_dropout.npz, float64); the forward-only call (no_grad in training mode,
    train.py:265-278) gives the same preds from the same seed."""
    g = golden("train_dropout.npz")
    fw, m = model_from_fixture("bandit5")
    A = int(fw["cfg"][2])
    pre = f"c{case}/"
    batch = {k: torch.from_numpy(g[pre + k]).float().cuda() for k in KEYS}
    batch["zeros"] = torch.from_numpy(g[pre + "zeros"]).float().cuda()
    opt = torch.from_numpy(g[pre + "optimal_actions"]).float().cuda()
    p, seed = float(g[pre + "p"]), int(g[pre + "seed"])
    m.train()
    loss, pred = _dropout_step(m, batch, opt, A, p, seed)
    ref_loss = float(g[pre + "loss"])
    assert abs(loss.item() - ref_loss) <= 1e-5 * abs(ref_loss)
    ref = g[pre + "preds"]
    assert (np.abs(pred.detach().cpu().numpy() - ref) <= 1e-5 * np.maximum(1, np.abs(ref))).all()
    for k, prm in m.named_parameters():
        if k.endswith("wte.weight"):
            continue
        r = g[pre + "grad/" + k]
        got = prm.grad.detach().cpu().numpy()
        got = got[:r.shape[0]] if k.endswith("wpe.weight") else got
        assert rel_err(got, r) <= 5 * GRAD_TOL, k
    with torch.no_grad():
        _, pred2 = _dropout_step(m, batch, opt, A, p, seed, grad=False)
    assert torch.equal(pred2, pred.detach())
    with torch.no_grad():
        _, pred3 = _dropout_step(m, batch, opt, A, p, seed + 1, grad=False)
    assert not torch.equal(pred3, pred.detach())   # another seed, other masks


@pytest.mark.parametrize("E,T", [(16, 38), (64, 103)])
def test_train_dropout_other_widths_vs_oracle(E, T):
    """Dropout at widths 16 / 64 (the widths whose p = 0 path runs the matrix-core kernels; with
    dropout the row kernels) against the float64 oracle with the same masks; windows with
    T % 4 != 0."""
    from models.net import Transformer
    from oracle import dpt_oracle_torch as OT
    from philox_np import dropout_keep
    A, L, B, C, sd, p, seed = 5, 2, 4, T - 1, 2, 0.2, 12345
    torch.manual_seed(E + T + 1)
    m = Transformer(dict(horizon=C, state_dim=sd, action_dim=A, n_layer=L, n_embd=E, n_head=1, dropout=p,
                         test=False))
    with torch.no_grad():
        for prm in m.parameters():
            prm.add_(0.05 * torch.randn_like(prm))
    w = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    m = m.cuda()
    rs = np.random.RandomState(E * 5 + T)
    hb = {"query_states": rs.randint(0, 10, (B, sd)).astype(np.float64),
          "context_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_actions": np.eye(A)[rs.randint(0, A, (B, C))],
          "context_next_states": rs.randint(0, 10, (B, C, sd)).astype(np.float64),
          "context_rewards": rs.normal(0.5, 0.5, (B, C, 1)), "optimal_actions": np.eye(A)[rs.randint(0, A, B)]}

    def drop(site):
        return torch.from_numpy(dropout_keep(seed, p, site, (B, T, T) if site % 3 == 1 else (B, T, E)))
    loss_ref, preds_ref, grads_ref = OT.grads(w, hb, L, sd, A, drop=drop)
    batch = {k: torch.tensor(hb[k], dtype=torch.float32, device="cuda") for k in KEYS}
    batch["zeros"] = torch.zeros((B, sd * sd + A + 1), device="cuda")
    opt = torch.tensor(hb["optimal_actions"], dtype=torch.float32, device="cuda")
    m.train()
    loss, pred = _dropout_step(m, batch, opt, A, p, seed)
    assert abs(loss.item() - loss_ref) <= 1e-5 * abs(loss_ref)
    assert (np.abs(pred.detach().cpu().numpy() - preds_ref) <= 1e-5 * np.maximum(1, np.abs(preds_ref))).all()
    for k, prm in m.named_parameters():
        if k.endswith("wte.weight"):
            continue
        assert rel_err(prm.grad.detach().cpu().numpy(), grads_ref[k]) <= 5 * GRAD_TOL, k


def test_train_dropout_through_the_model_forward():
    """Transformer.forward in training mode with dropout > 0 (the reference's --dropout flag):
    seeds come from torch's CUDA generator -- the same manual_seed, the same preds; a second call,
    new masks -- and eval mode applies none (equal to the p = 0 model's preds)."""
    g = golden("train_grads.npz")
    _, m = model_from_fixture("bandit5")
    batch, _ = batch_from(g, "bandit5")
    m.dropout = 0.3
    m.train()
    torch.manual_seed(3)
    a = m(batch).detach()
    b = m(batch).detach()
    torch.manual_seed(3)
    c = m(batch).detach()
    assert torch.equal(a, c) and not torch.equal(a, b)
    m.eval()
    with torch.no_grad():
        e = m(batch)
    m.dropout = 0.0
    with torch.no_grad():
        f = m(batch)
    assert torch.equal(e, f)


def test_dropout_leaves_the_cpu_stream_alone():
    """Dropout seeds come from the CUDA generator (models/net.py _dropout_seed), as the reference's
    dropout masks do, so the CPU stream that drives the DataLoader shuffle (train.py:203,249) and the
    per-item context permutation (dataset.py:85) is the same with and without dropout: a shuffled
    DataLoader's batch order over two epochs, with a dropout training forward after every batch,
    equals the order with dropout 0.  torch.manual_seed reproduces the seeds."""
    from models import net
    g = golden("train_grads.npz")
    _, m = model_from_fixture("bandit5")
    batch, _ = batch_from(g, "bandit5")
    m.train()
    orders = []
    for p in (0.0, 0.2):
        m.dropout = p
        torch.manual_seed(11)
        dl = torch.utils.data.DataLoader(torch.arange(64), batch_size=8, shuffle=True)
        order = []
        for _ in range(2):
            for idx in dl:
                order.append(idx.clone())
                m(batch)
        orders.append(torch.cat(order))
    assert torch.equal(orders[0], orders[1])
    torch.manual_seed(5)
    s1, s2 = net._dropout_seed(), net._dropout_seed()
    torch.manual_seed(5)
    assert net._dropout_seed() == s1 and s1 != s2


def _width_model(E, L, H, seed):
    from models.net import Transformer
    torch.manual_seed(seed)
    m = Transformer(dict(horizon=H, state_dim=1, action_dim=5, n_layer=L, n_embd=E, n_head=1, dropout=0.0,
                         test=True)).cuda().eval()
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.05 * torch.randn_like(p))
    return m


@pytest.mark.parametrize("E,L,bern,sample", [(16, 3, False, True), (48, 2, False, True), (64, 4, True, True),
                                             (64, 2, False, False), (32, 2, False, True), (18, 2, False, True),
                                             (128, 2, False, True)])
def test_generic_width_rollout_vs_oracle(E, L, bern, sample):
    """dpt_rollout_bandit_generic (the bandit online loop at any width: exact K/V-cache decode, one
    step for all tasks at a time) against the float64 oracle's re-forward-every-step rollout fed the
    same draws: logits within 1e-5 at every step, actions / rewards / arm values exactly.  Widths on
    the row kernels (18, 48, 128) and on the matrix-core forms (16, 32, 64); the float4 attention
    (E % 4 == 0) and the scalar one (18); Gaussian and Bernoulli rewards, sampling and greedy; 37
    tasks (a partial row block)."""
    from dpt_hip import train as tr
    from oracle import dpt_oracle as O
    N, H = 37, 40
    m = _width_model(E, L, H, E + L)
    W = O.split_weights({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}, L)
    rs = np.random.RandomState(E * 3 + L)
    means = rs.uniform(0, 1, (N, 5))
    u = rs.uniform(size=(H, N))
    g = rs.uniform(size=(H, N)) if bern else rs.normal(size=(H, N))
    out = tr.rollout_bandit_generic(m, means, H, 0.3, sample, 1 if bern else 0, uniforms=u, noise=g,
                                    want_logits=True)
    ref = O.bandit_online_rollout(W, means, H, 0.3, u, g, sample=sample, bernoulli=bern)
    lg = out["logits"].cpu().numpy()
    assert (np.abs(lg - ref["logits"]) <= 1e-5 * np.maximum(1, np.abs(ref["logits"]))).all()
    assert np.array_equal(out["actions"].cpu().numpy(), ref["actions"])
    assert np.array_equal(out["rewards"].cpu().numpy(), ref["rewards"])
    assert np.array_equal(out["arm_value"].cpu().numpy().T, ref["cum_means"])


def test_generic_width_rollout_equals_fused_kernel_at_width_32():
    """At width 32 the generic-width rollout and the fused kernel (dpt_rollout_bandit) run the same
    loop: with the same Philox draws (seed, counter, global task ids) the actions agree; with
    injected draws over 300 tasks x 80 steps every task agrees up to its first step whose uniform
    lies within 1e-5 of a cdf edge (where the two fp32 summation orders may choose differently),
    with logits within 1e-5 of each other up to that step."""
    from dpt_hip import train as tr
    N, H, L = 300, 80, 4
    m = _width_model(32, L, H, 7)
    rs = np.random.RandomState(3)
    means = rs.uniform(0, 1, (N, 5))
    a = tr.rollout_bandit_generic(m, means[:16], 12, 0.3, True, seed=99, first_task=1000, counter=5)
    b = m.device_model().rollout_bandit(means[:16], 12, 0.3, True, seed=99, first_task=1000, counter=5)
    assert np.array_equal(a["rewards"].cpu().numpy(), b["rewards"].cpu().numpy())   # same Philox draws
    u, g = rs.uniform(size=(H, N)), rs.normal(size=(H, N))
    a = tr.rollout_bandit_generic(m, means, H, 0.3, True, uniforms=u, noise=g, want_logits=True)
    b = m.device_model().rollout_bandit(means, H, 0.3, True, uniforms=u, noise=g, want_logits=True)
    la, lb = a["logits"].cpu().numpy(), b["logits"].cpu().numpy()
    aa, ab = a["actions"].cpu().numpy(), b["actions"].cpu().numpy()
    ra, rb = a["rewards"].cpu().numpy(), b["rewards"].cpu().numpy()
    for i in range(N):
        diff = np.nonzero(aa[i] != ab[i])[0]
        n = int(diff[0]) if diff.size else H
        if n < H:  # the first disagreement must be a near-tie of the draw with the cdf
            p = np.exp(lb[n, i].astype(np.float64) - lb[n, i].max())
            cdf = np.cumsum(p / p.sum())
            assert np.abs(cdf[:-1] - u[n, i]).min() < 1e-5, (i, n)
        k = min(n + 1, H)
        assert (np.abs(la[:k, i] - lb[:k, i]) <= 1e-5 * np.maximum(1, np.abs(lb[:k, i]))).all(), i
        assert np.array_equal(ra[i, :n], rb[i, :n]), i


def test_generic_width_rollout_through_eval_bandit():
    """eval_bandit.deploy_online_vec with a width-64 controller takes the generic-width rollout
    (one call) and returns the per-step loop's cum_means (fused=False: the reference's loop, the
    whole window re-forwarded every step) for the same draws."""
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    from dpt_hip import train as tr
    n, H = 9, 24
    m = _width_model(64, 3, H, 5)
    rs = np.random.RandomState(8)
    means = rs.uniform(0, 1, (n, 5))
    u, g = rs.uniform(size=(H, n)), rs.normal(size=(H, n))
    calls = []
    real = tr.rollout_bandit_generic

    def spy(*a, **k):
        calls.append(1)
        return real(*a, **k)
    tr.rollout_bandit_generic = spy
    try:
        vec = BanditEnvVec([BanditEnv(mu, H, var=0.3) for mu in means])
        cm = eval_bandit.deploy_online_vec(vec, BanditTransformerController(m, sample=True, batch_size=n), H,
                                           uniforms=u, noise=g)
    finally:
        tr.rollout_bandit_generic = real
    vec = BanditEnvVec([BanditEnv(mu, H, var=0.3) for mu in means])
    cm_ref = eval_bandit.deploy_online_vec(vec, BanditTransformerController(m, sample=True, batch_size=n), H,
                                           uniforms=u, noise=g, fused=False)
    assert calls == [1]
    assert np.array_equal(cm, cm_ref)
