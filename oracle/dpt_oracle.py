"""CPU oracle for the DPT rollout / in-context-eval hot path.  TEST INFRASTRUCTURE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the CHECKER (or the CPU timing
baseline) — never as the thing measured or shipped.  The product path
(``decision-pretrained-transformer_amd/``) must never import it.

Parity status: PINNED.  Every function below is checked against golden vectors
recorded from the reference itself (``tests/golden/*.npz``, produced by
``tests/golden/gen_golden.py`` importing /root/reference on CPU):
bit-exact for env transitions / indices / rewards, ``<= 1e-5`` on fp32 logits.

Reference = titanium-47/decision-pretrained-transformer (citations are
``path:line`` relative to its root).  The transformer arithmetic lives in the
third-party ``transformers`` package (pinned 4.5.1 by requirements.txt:1,
5.15.0 installed here); its GPT-2 block is restated from
``transformers/models/gpt2/modeling_gpt2.py`` (GPT2Block.forward,
GPT2Attention.forward, GPT2MLP.forward) and ``activations.py`` (NewGELU).
"""
import itertools
import math

import numpy as np

LN_EPS = 1e-5  # GPT2Config.layer_norm_epsilon default

# ----------------------------------------------------------------------------- environments


def bandit_reward(means, action, g, var):
    """Gaussian bandit reward, fp64, two roundings, no FMA.

    envs/bandit_env.py:56-64: ``r = means[a] + np.random.normal(0, var)`` and
    legacy ``normal(0, s) == 0.0 + s * g`` (pinned by gen_golden.DrawRecorder).
    """
    means = np.asarray(means, np.float64)
    a = np.asarray(action)
    noise = 0.0 + np.float64(var) * np.asarray(g, np.float64)
    return means[np.arange(means.shape[0]), a] + noise


def gpu_bandit_reward_f32(means32, action, g32, var):
    """GPUBanditEnv.transit (envs/gpu_bandit_env.py:53-63): fp32 torch ops
    ``means[ar, argmax(us)] + torch.randn(N) * var``: the python-float ``var`` is cast to fp32,
    then one fp32 multiply and one fp32 add (two roundings)."""
    m = np.asarray(means32, np.float32)[np.arange(len(action)), np.asarray(action)]
    return m + np.asarray(g32, np.float32) * np.float32(var)


def bernoulli_reward(means, action, u):
    """Bernoulli bandit: ``torch.bernoulli(mean)`` == ``u < mean`` (envs/gpu_bandit_env.py:58-61)."""
    means = np.asarray(means, np.float64)
    m = means[np.arange(means.shape[0]), np.asarray(action)]
    return (np.asarray(u, np.float64) < m).astype(np.float64)


def arm_value(means, action):
    """``get_arm_value(onehot) = sum(means * onehot) = means[a]`` (envs/bandit_env.py:151-153)."""
    means = np.asarray(means, np.float64)
    return means[np.arange(means.shape[0]), np.asarray(action)]


def linear_means(arms, theta):
    """``means = arms @ theta`` per env (envs/bandit_env.py:158-161).

    Kept as the same per-env numpy GEMV call: OpenBLAS evaluates the d=2 dot as
    ``fma(a0, t0, a1*t1)`` (measured on the golden vectors), so a batched matmul
    or a plain two-rounding sum is NOT bit-identical.  Task setup, host-side.
    """
    arms = np.asarray(arms, np.float64)
    return np.stack([arms @ t for t in np.asarray(theta, np.float64)])


def perm_table():
    """All 120 action permutations in ``itertools.permutations`` order (envs/darkroom_env.py:97-99)."""
    return np.array(list(itertools.permutations(range(5))), dtype=np.int64)


def darkroom_transit(state, action, goal, dim=10, perm=None):
    """Vectorised DarkRoom transition (envs/darkroom_env.py:37-55; permuted :100-103).

    action 0:+x 1:-x 2:+y 3:-y 4:stay, clip to [0, dim-1], reward 1 iff next == goal.
    """
    s = np.array(state, dtype=np.int64, copy=True)
    a = np.asarray(action, dtype=np.int64)
    if perm is not None:
        a = np.asarray(perm, dtype=np.int64)[np.arange(len(a)), a]
    s[:, 0] += (a == 0).astype(np.int64) - (a == 1).astype(np.int64)
    s[:, 1] += (a == 2).astype(np.int64) - (a == 3).astype(np.int64)
    s = np.clip(s, 0, dim - 1)
    r = np.all(s == np.asarray(goal), axis=1).astype(np.int64)
    return s, r


def darkroom_opt_action(state, goal, perm=None):
    """Greedy x-then-y expert (envs/darkroom_env.py:69-82); permuted inverse map :105-111."""
    s = np.asarray(state)
    g = np.asarray(goal)
    a = np.full(len(s), 4, dtype=np.int64)
    a = np.where(s[:, 1] > g[:, 1], 3, a)
    a = np.where(s[:, 1] < g[:, 1], 2, a)
    a = np.where(s[:, 0] > g[:, 0], 1, a)
    a = np.where(s[:, 0] < g[:, 0], 0, a)
    if perm is not None:
        perm = np.asarray(perm)
        a = np.argmax(perm == a[:, None], axis=1)
    return a


# ----------------------------------------------------------------------------- model


def split_weights(w, n_layer):
    """Named views of a reference ``Transformer.state_dict()`` (models/net.py:25-39)."""
    g = lambda k: np.asarray(w[k])  # noqa: E731
    layers = []
    for i in range(n_layer):
        p = f"transformer.h.{i}."
        layers.append(dict(
            ln1_g=g(p + "ln_1.weight"), ln1_b=g(p + "ln_1.bias"),
            attn_w=g(p + "attn.c_attn.weight"), attn_b=g(p + "attn.c_attn.bias"),
            proj_w=g(p + "attn.c_proj.weight"), proj_b=g(p + "attn.c_proj.bias"),
            ln2_g=g(p + "ln_2.weight"), ln2_b=g(p + "ln_2.bias"),
            fc_w=g(p + "mlp.c_fc.weight"), fc_b=g(p + "mlp.c_fc.bias"),
            mp_w=g(p + "mlp.c_proj.weight"), mp_b=g(p + "mlp.c_proj.bias")))
    return dict(emb_w=g("embed_transition.weight"), emb_b=g("embed_transition.bias"),
                wpe=g("transformer.wpe.weight"), lnf_g=g("transformer.ln_f.weight"),
                lnf_b=g("transformer.ln_f.bias"), head_w=g("pred_actions.weight"),
                head_b=g("pred_actions.bias"), layers=layers)


def pack_tokens(query, cs, ca, cn, cr, action_dim, state_dim):
    """Token packing of ``Transformer.forward`` (models/net.py:41-54).

    position 0 = [query, 0_A, 0_sd, 0]; position 1+j = [s_j, a_j, s'_j, r_j].
    """
    n = query.shape[0]
    q = np.concatenate([np.asarray(query, np.float64)[:, None, :],
                        np.zeros((n, 1, action_dim + state_dim + 1))], axis=2)
    ctx = np.concatenate([cs, ca, cn, np.asarray(cr).reshape(n, -1, 1)], axis=2)
    return np.concatenate([q, np.asarray(ctx, np.float64)], axis=1)


def layer_norm(x, g, b):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return (x - mu) / np.sqrt(var + LN_EPS) * g + b


def gelu_new(x):
    """NewGELUActivation (transformers/activations.py:65)."""
    return 0.5 * x * (1.0 + np.tanh(math.sqrt(2.0 / math.pi) * (x + 0.044715 * x ** 3)))


def gpt2_hidden(W, seq, dtype=np.float64):
    """Embed + GPT-2 stack + ln_f over packed tokens ``seq`` (N, T, F) -> (N, T, E).

    models/net.py:52-54 (embed_transition, inputs_embeds) and the GPT2Model
    forward: h = emb + wpe[0:T]; per block h += attn(ln_1 h); h += mlp(ln_2 h);
    ln_f.  One head (net.py:29 forces n_head=1) -> scale 1/sqrt(E); causal.
    """
    cast = lambda a: np.asarray(a, dtype)  # noqa: E731
    x = cast(seq) @ cast(W["emb_w"]).T + cast(W["emb_b"])
    T = x.shape[1]
    E = x.shape[2]
    x = x + cast(W["wpe"])[:T]
    mask = np.triu(np.ones((T, T), dtype=bool), 1)
    scale = dtype(E ** -0.5) if dtype is not np.float64 else E ** -0.5
    for Lw in W["layers"]:
        h = layer_norm(x, cast(Lw["ln1_g"]), cast(Lw["ln1_b"]))
        qkv = h @ cast(Lw["attn_w"]) + cast(Lw["attn_b"])
        q, k, v = qkv[..., :E], qkv[..., E:2 * E], qkv[..., 2 * E:]
        s = (q @ np.swapaxes(k, 1, 2)) * scale
        s = np.where(mask, -np.inf, s)
        s = s - s.max(-1, keepdims=True)
        p = np.exp(s)
        p = p / p.sum(-1, keepdims=True)
        a = p @ v
        x = x + (a @ cast(Lw["proj_w"]) + cast(Lw["proj_b"]))
        h = layer_norm(x, cast(Lw["ln2_g"]), cast(Lw["ln2_b"]))
        m = gelu_new(h @ cast(Lw["fc_w"]) + cast(Lw["fc_b"]))
        x = x + (m @ cast(Lw["mp_w"]) + cast(Lw["mp_b"]))
    return layer_norm(x, cast(W["lnf_g"]), cast(W["lnf_b"]))


def transformer_forward(W, query, cs, ca, cn, cr, test=True, dtype=np.float64):
    """``Transformer.forward`` (models/net.py:41-60): last position (test) or positions 1..T-1."""
    A = W["head_w"].shape[0]
    sd = np.asarray(query).shape[1]
    seq = pack_tokens(np.asarray(query), np.asarray(cs), np.asarray(ca), np.asarray(cn),
                      np.asarray(cr), A, sd)
    hdn = gpt2_hidden(W, seq, dtype)
    cast = lambda a: np.asarray(a, dtype)  # noqa: E731
    preds = hdn @ cast(W["head_w"]).T + cast(W["head_b"])
    return preds[:, -1, :] if test else preds[:, 1:, :]


# ----------------------------------------------------------------------------- action selection


def softmax_f32(logits, temp=None):
    """``scipy.special.softmax`` on float32 logits (ctrls/ctrl_bandit.py:436; ctrl_darkroom.py:51).

    max-shift, exp, sum and divide all stay in float32 (scipy 1.15 keeps dtype).
    """
    x = np.asarray(logits, np.float32)
    if temp is not None:
        x = x / np.float32(temp) if isinstance(temp, np.floating) else x / temp
    e = np.exp(x - x.max(-1, keepdims=True))
    return e / e.sum(-1, keepdims=True)


def choice_from_uniform(p, u):
    """numpy legacy ``RandomState.choice(A, p=p)`` given its one uniform draw ``u``:
    ``cdf = cumsum(float64(p)); cdf /= cdf[-1]; idx = searchsorted(cdf, u, 'right')``.
    Pinned against the real call by tests/golden/gen_golden.py (DrawRecorder)."""
    p = np.asarray(p, np.float64)
    cdf = np.cumsum(p, axis=-1)
    cdf = cdf / cdf[..., -1:]
    u = np.asarray(u, np.float64)
    return (cdf <= u[..., None]).sum(-1)


def boundary_margin(p, u):
    """Distance of ``u`` to the nearest interior cdf edge (flags near-tie samples)."""
    p = np.asarray(p, np.float64)
    cdf = np.cumsum(p, axis=-1)
    cdf = cdf / cdf[..., -1:]
    return np.abs(cdf[..., :-1] - np.asarray(u, np.float64)[..., None]).min(-1)


def select_actions(logits, u=None, sample=True, temp=None):
    """BanditTransformerController.act_numpy_vec / DarkroomTransformerController.act
    selection (ctrls/ctrl_bandit.py:435-443, ctrls/ctrl_darkroom.py:48-62)."""
    if not sample:
        return np.argmax(np.asarray(logits, np.float32), axis=-1)
    return choice_from_uniform(softmax_f32(logits, temp), u)


# ----------------------------------------------------------------------------- rollouts


def bandit_online_rollout(W, means, H, var, u, g, sample=True, dtype=np.float64,
                          bernoulli=False):
    """evals/eval_bandit.py:56-103 ``deploy_online_vec`` with the DPT controller
    (ctrls/ctrl_bandit.py:383-444) and ``BanditEnvVec.deploy`` (envs/bandit_env.py:125-149).

    Exactly the reference algorithm: the whole window is re-forwarded at every
    step.  ``u``/``g`` (H, N) are the injected per-step uniforms / normals.
    Returns cum_means (H, N) fp64, actions (N, H), rewards (N, H) fp64, logits (H, N, A).
    """
    means = np.asarray(means, np.float64)
    N, A = means.shape
    ca = np.zeros((N, H, A))
    cr = np.zeros((N, H, 1))
    ones = np.ones((N, H, 1))
    acts = np.zeros((N, H), np.int64)
    cum = np.zeros((H, N))
    logs = np.zeros((H, N, A), np.float32)
    for h in range(H):
        lg = transformer_forward(W, np.ones((N, 1)), ones[:, :h], ca[:, :h], ones[:, :h],
                                 cr[:, :h], dtype=dtype).astype(np.float32)
        logs[h] = lg
        a = select_actions(lg, u[h] if sample else None, sample)
        if bernoulli:
            r = bernoulli_reward(means, a, g[h])
        else:
            r = bandit_reward(means, a, g[h], var)
        ca[np.arange(N), h, a] = 1.0
        cr[:, h, 0] = r
        acts[:, h] = a
        cum[h] = arm_value(means, a)
    return dict(cum_means=cum, actions=acts, rewards=cr[..., 0], logits=logs)


def darkroom_online_rollout(W, goals, Heps, H, horizon, u, sample=True, perm=None,
                            dim=10, dtype=np.float64):
    """evals/eval_darkroom.py:20-84 ``deploy_online_vec`` with
    DarkroomTransformerController (ctrls/ctrl_darkroom.py:23-66) and
    ``DarkroomEnvVec.deploy_eval`` (envs/darkroom_env.py:151-175).

    Episode i < H/horizon sees the first i episodes; later episodes see the last
    H/horizon episodes (shift-append :75-82).  Returns (N, Heps) returns.
    """
    goals = np.asarray(goals)
    N = goals.shape[0]
    R = H // horizon
    cs = np.zeros((N, R, horizon, 2))
    ca = np.zeros((N, R, horizon, 5))
    cn = np.zeros((N, R, horizon, 2))
    cr = np.zeros((N, R, horizon, 1))
    rets = np.zeros((N, Heps), np.int64)
    logs, acts = [], []
    for ep in range(Heps):
        nctx = min(ep, R)
        if ep < R:
            b = [x[:, :nctx].reshape(N, -1, x.shape[-1]) for x in (cs, ca, cn, cr)]
        else:
            b = [x.reshape(N, -1, x.shape[-1]) for x in (cs, ca, cn, cr)]
        s = np.zeros((N, 2), np.int64)
        es, ea, en, er = [], [], [], []
        for t in range(horizon):
            lg = transformer_forward(W, s.astype(np.float64), *b, dtype=dtype).astype(np.float32)
            logs.append(lg)
            a = select_actions(lg, u[ep, t] if sample else None, sample,
                               temp=1.0 if sample else None)
            ns, r = darkroom_transit(s, a, goals, dim, perm)
            acts.append(a)
            es.append(s.copy())
            ea.append(np.eye(5)[a])
            en.append(ns.copy())
            er.append(r)
            s = ns
        es, ea, en, er = (np.stack(x, 1) for x in (es, ea, en, er))
        rets[:, ep] = er.sum(-1)
        new = (es.astype(np.float64), ea, en.astype(np.float64), er[..., None].astype(np.float64))
        if ep < R:
            for buf, v in zip((cs, ca, cn, cr), new):
                buf[:, ep] = v
        else:
            for buf, v in zip((cs, ca, cn, cr), new):
                buf[:, :-1] = buf[:, 1:].copy()
                buf[:, -1] = v
    return dict(returns=rets, logits=np.stack(logs), actions=np.stack(acts, 1))


def darkroom_offline_episode(W, goals, ctx, horizon, u, sample=True, perm=None, dim=10, dtype=np.float64):
    """One ``DarkroomEnvVec.deploy_eval`` episode of the DPT controller on a FIXED context
    (evals/eval_darkroom.py:124-189 ``offline``: ``lnr.set_batch(batch)`` then
    ``vec_env.deploy_eval``; envs/darkroom_env.py:151-175): from (0, 0), every step forwards
    [query = current state | context], selects (sampled with temp 1.0, or argmax) and steps the
    grid.  ctx = (cs, ca, cn, cr) with cr (N, C, 1).  Returns rewards (N, horizon) int."""
    goals = np.asarray(goals)
    N = goals.shape[0]
    s = np.zeros((N, 2), np.int64)
    rews = np.zeros((N, horizon), np.int64)
    for t in range(horizon):
        lg = transformer_forward(W, s.astype(np.float64), *ctx, dtype=dtype).astype(np.float32)
        a = select_actions(lg, u[t] if sample else None, sample, temp=1.0 if sample else None)
        s, r = darkroom_transit(s, a, goals, dim, perm)
        rews[:, t] = r
    return rews


def darkroom_opt_returns(goals, horizon, perm=None, dim=10):
    """The expert leg of the offline eval (evals/eval_darkroom.py:146-150: DarkroomOptPolicy
    deployed per env, ctrls/ctrl_darkroom.py:10-20): sum of rewards over one episode."""
    goals = np.asarray(goals)
    s = np.zeros((goals.shape[0], 2), np.int64)
    tot = np.zeros(goals.shape[0], np.int64)
    for _ in range(horizon):
        s, r = darkroom_transit(s, darkroom_opt_action(s, goals, perm), goals, dim, perm)
        tot += r
    return tot


def regret_curves(opt, lnr):
    """Suboptimality + cumulative regret mean/SEM over tasks (evals/eval_bandit.py:169-178).

    opt, lnr: (N, H) per-step arm values.  SEM uses ddof=1 (scipy.stats.sem default).
    """
    diff = np.asarray(opt, np.float64) - np.asarray(lnr, np.float64)
    n = diff.shape[0]
    cr = np.cumsum(diff, axis=1)
    sem = lambda x: x.std(0, ddof=1) / np.sqrt(n)  # noqa: E731
    return dict(subopt_mean=diff.mean(0), subopt_sem=sem(diff),
                regret_mean=cr.mean(0), regret_sem=sem(cr))


def rollin_bandit(means, cov, dirichlet, rand_index, u, g, var):
    """collect_data.py:23-53 behaviour policy + H transits, draws injected.

    p = (1 - cov) * Dir(1_A) + cov * e_rand; each step i ~ choice(A, p); r = means[i] + var*g.
    """
    means = np.asarray(means, np.float64)
    A = means.shape[0]
    probs2 = np.zeros(A)
    probs2[int(rand_index)] = 1.0
    p = (1 - cov) * np.asarray(dirichlet, np.float64) + cov * probs2
    idx = choice_from_uniform(np.broadcast_to(p, (len(u), A)), np.asarray(u))
    us = np.eye(A)[idx]
    rs = means[idx] + (0.0 + var * np.asarray(g, np.float64))
    return np.ones((len(u), 1)), us, np.ones((len(u), 1)), rs


# ----------------------------------------------------------------------------- classical baselines


def policy_action(policy, acts_ctx, rews_ctx, A, online=True, c=1.0, ts=None, ts_g=None, arms=None,
                  first_u_idx=None):
    """One decision of a classical controller from its context (fp64 numpy, the reference's
    arithmetic).  acts_ctx (N, h) int, rews_ctx (N, h) float64.

    emp: ctrls/ctrl_bandit.py:89-118; ucb :348-380; lcb :286-314; thompson :184-236
    (sample=True, posterior normals ts_g (N, A)); linucb :488-528 (first_u_idx (N) for h=0).
    """
    N, h = acts_ctx.shape
    if policy == "linucb":
        if h < 1:
            return np.asarray(first_u_idx)
        out = np.zeros(N, np.int64)
        for i in range(N):
            X = arms[acts_ctx[i]]
            cov = np.eye(arms.shape[1]) + X.T @ X
            cinv = np.linalg.inv(cov)
            theta = (cinv @ X.T @ rews_ctx[i][:, None]).flatten()
            best, bi = -np.inf, None
            for k, arm in enumerate(arms):
                v = theta @ arm + c * np.sqrt(arm @ cinv @ arm)
                if v > best:
                    best, bi = v, k
            out[i] = bi
        return out
    b = np.zeros((N, A))
    counts = np.zeros((N, A))
    for i in range(N):
        for k in range(A):
            r = rews_ctx[i][acts_ctx[i] == k]
            b[i, k] = np.sum(r)
            counts[i, k] = len(r)
    if policy == "thompson":
        var, pm, pv = ts["std"] ** 2, ts["prior_mean"], ts["prior_var"]
        means = np.ones((N, A)) * pm
        variances = np.ones((N, A)) * pv
        arm_means = np.zeros((N, A))
        for i in range(N):
            for k in range(A):
                if counts[i, k] > 0:
                    arm_means[i, k] = np.mean(rews_ctx[i][acts_ctx[i] == k])
        with np.errstate(divide="ignore", invalid="ignore"):
            w = var / (var + counts * pv)
            new_mean = w * pm + (1 - w) * arm_means
            new_var = 1 / (1 / pv + counts / var)
        mask = counts > 0
        means[mask] = new_mean[mask]
        variances[mask] = new_var[mask]
        return np.argmax(means + np.sqrt(variances) * ts_g, axis=-1)
    b_mean = b / np.maximum(1, counts)
    if policy in ("ucb", "lcb"):
        bons = c / np.maximum(1, np.sqrt(counts))
        b_mean = b_mean + bons if policy == "ucb" else b_mean - bons
    i = np.argmax(b_mean, axis=-1)
    if policy == "ucb" or (policy == "emp" and online):
        j = np.argmin(counts, axis=-1)
        mask = counts[np.arange(N), j] == 0
        i[mask] = j[mask]
    return i


def bandit_policy_rollout(policy, means, H, var, g, ctx_actions=None, ctx_rewards=None, bernoulli=False, **kw):
    """evals/eval_bandit.py:56-103 with a classical controller; draws injected.
    g (H, N): reward normals, or uniforms with bernoulli=True (BanditEnv.transit's Binomial(1, mean),
    envs/bandit_env.py:56-64, as u < mean).  ctx_actions / ctx_rewards (N, C): a prefix context the
    controller sees before the first step (set_batch_numpy_vec, evals/eval_bandit.py:214-301).
    kw: online, c, ts (dict std/prior_mean/prior_var), ts_g (H, N, A), arms, first_u_idx."""
    means = np.asarray(means, np.float64)
    N, A = means.shape
    C = 0 if ctx_actions is None else np.asarray(ctx_actions).shape[1]
    acts = np.zeros((N, C + H), np.int64)
    rews = np.zeros((N, C + H))
    if C:
        acts[:, :C] = ctx_actions
        rews[:, :C] = ctx_rewards
    ts_g = kw.pop("ts_g", None)
    for h in range(H):
        n = C + h
        a = policy_action(policy, acts[:, :n], rews[:, :n], A, ts_g=None if ts_g is None else ts_g[h], **kw)
        acts[:, n] = a
        rews[:, n] = bernoulli_reward(means, a, g[h]) if bernoulli else bandit_reward(means, a, g[h], var)
    acts, rews = acts[:, C:], rews[:, C:]
    return dict(actions=acts, rewards=rews, cum_means=np.stack([arm_value(means, acts[:, h]) for h in range(H)]))
