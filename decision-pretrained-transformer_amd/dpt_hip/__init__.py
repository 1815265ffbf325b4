"""Device runtime of the MI355X DPT hot path: torch tensors in, libdpt_hip.so kernels out.

PyTorch-ROCm is plumbing here (device memory, the current HIP stream); every
computation below is a hand-written gfx950 kernel behind the C ABI in
include/dpt_hip.h.  There is deliberately no CPU implementation: calling any
of these without a GPU raises.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (BANDIT_BERNOULLI, BANDIT_F32, BANDIT_GAUSSIAN, STREAM_REWARD, STREAM_ROLLIN,  # noqa: F401
                   STREAM_SELECT, EpisodeEndedError)

E = 32


def device():
    """The device the hot path runs on (``cuda`` == HIP on ROCm)."""
    if not torch.cuda.is_available():
        raise RuntimeError("the DPT HIP path needs a ROCm GPU (torch.cuda.is_available() is False)")
    _lib.load()
    return torch.device("cuda", torch.cuda.current_device())


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _dev(x, dtype, dev=None):
    dev = dev or device()
    if isinstance(x, torch.Tensor):
        return x.to(device=dev, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=dev)


def next_seed():
    """64-bit Philox key drawn from numpy's global RNG (so ``np.random.seed`` governs
    the run, as it does in the reference: eval.py:64-71, collect_data.py:352)."""
    return int(np.random.randint(0, 2 ** 62, dtype=np.int64))


# ----------------------------------------------------------------------------- weights

def layer_param_names(i):
    p = f"transformer.h.{i}."
    return [p + n for n in ("ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias",
                            "attn.c_proj.weight", "attn.c_proj.bias", "ln_2.weight", "ln_2.bias",
                            "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias")]


def pack_weights(sd, n_layer):
    """Flatten a reference ``Transformer.state_dict()`` into the dpt_hip.h blob order.

    nn.Linear weights (embed_transition, pred_actions) are stored [out][in] by
    torch and transposed here; GPT-2 Conv1D weights are already [in][out].
    """
    def t(k):
        v = sd[k]
        return v.detach().to("cpu", torch.float32) if isinstance(v, torch.Tensor) else torch.as_tensor(v, dtype=torch.float32)

    parts = [t("embed_transition.weight").t(), t("embed_transition.bias"), t("transformer.wpe.weight")]
    for i in range(n_layer):
        parts += [t(k) for k in layer_param_names(i)]
    parts += [t("transformer.ln_f.weight"), t("transformer.ln_f.bias"),
              t("pred_actions.weight").t(), t("pred_actions.bias")]
    return torch.cat([p.contiguous().reshape(-1) for p in parts])


class DeviceModel:
    """Owns one ``dpt_model`` handle (the packed fp32 weights on the GPU)."""

    def __init__(self, state_dict, n_layer, state_dim, action_dim, n_positions, n_embd=E):
        self.desc = _lib.ModelDesc(n_layer, n_embd, state_dim, action_dim, n_positions)
        numel = ctypes.c_int64()
        _lib.call("dpt_weights_numel", ctypes.byref(self.desc), ctypes.byref(numel))
        blob = pack_weights(state_dict, n_layer)
        if blob.numel() != numel.value:
            raise ValueError(f"packed weights {blob.numel()} != expected {numel.value}")
        dev = device()
        blob_d = blob.to(dev)
        h = ctypes.c_void_p()
        _lib.call("dpt_model_create", ctypes.byref(self.desc), _p(blob_d), ctypes.byref(h))
        torch.cuda.current_stream().synchronize()
        self._h = h
        self.n_layer, self.state_dim, self.action_dim = n_layer, state_dim, action_dim
        self.n_positions = n_positions
        self.F = 2 * state_dim + action_dim + 1

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().dpt_model_free(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    def kv_numel(self, N, max_pos):
        n = ctypes.c_int64()
        _lib.call("dpt_kvcache_numel", self._h, int(N), int(max_pos), ctypes.byref(n))
        return n.value

    def forward_window(self, query, cs=None, ca=None, cn=None, cr=None, out_mode=0):
        """Transformer.forward (models/net.py:41-60) on device. Returns (N,A) or (N,C,A)."""
        dev = device()
        q = _dev(query, torch.float32, dev)
        N = q.shape[0]
        C = 0 if cs is None else int(cs.shape[1])
        if C:
            cs_, ca_, cn_ = (_dev(x, torch.float32, dev) for x in (cs, ca, cn))
            cr_ = _dev(cr, torch.float32, dev).reshape(N, C)
        else:
            cs_ = ca_ = cn_ = cr_ = None
        out = torch.empty((N, self.action_dim) if out_mode == 0 else (N, C, self.action_dim),
                          dtype=torch.float32, device=dev)
        if N == 0 or (out_mode == 1 and C == 0):  # empty batch / no context rows: nothing to run
            return out
        ws = (None if C + 1 <= self.prefill_max_window()
              else torch.empty(self.kv_numel(N, C + 1), dtype=torch.float32, device=dev))
        _lib.call("dpt_forward_window", self._h, _p(q), _p(cs_), _p(ca_), _p(cn_), _p(cr_), N, C,
                  int(out_mode), _p(out), _p(ws), _stream())
        return out

    def prefill_max_window(self):
        """Longest window dpt_forward_window runs as one MFMA prefill (0 when switched off)."""
        n = ctypes.c_int32()
        _lib.call("dpt_prefill_max_window", self._h, ctypes.byref(n))
        return n.value

    def decode_step(self, kv, max_pos, pos, token):
        token = _dev(token, torch.float32)
        N = token.shape[0]
        logits = torch.empty((N, self.action_dim), dtype=torch.float32, device=token.device)
        _lib.call("dpt_decode_step", self._h, _p(kv), N, int(max_pos), int(pos), _p(token), _p(logits),
                  _stream())
        return logits

    def rollout_bandit(self, means, H, var, sample=True, bandit_type=BANDIT_GAUSSIAN, seed=0,
                       first_task=0, uniforms=None, noise=None, want_logits=False, counter=0, kvcache=None):
        """Fused online bandit rollout (evals/eval_bandit.py:56-103) on device.

        Step h draws at Philox counter ``counter + h`` (global task id first_task + i),
        the counters the per-step path's selects would consume from ``counter`` on.
        ``kvcache``, optional: the caller's fp32 device workspace (at least ``kv_numel(N, H)``
        elements, e.g. a view into a larger allocation); by default one is allocated.

        Returns dict of device tensors: actions (N,H) int32, rewards (N,H) f64,
        arm_value (N,H) f64 (= cum_means.T), logits (H,N,A) f32 if requested.
        """
        dev = device()
        means_d = _dev(means, torch.float64, dev)
        N, A = means_d.shape
        H = int(H)
        out = dict(actions=torch.empty((N, H), dtype=torch.int32, device=dev),
                   rewards=torch.empty((N, H), dtype=torch.float64, device=dev),
                   arm_value=torch.empty((N, H), dtype=torch.float64, device=dev))
        out["logits"] = (torch.empty((H, N, A), dtype=torch.float32, device=dev) if want_logits else None)
        if N == 0 or H == 0:  # no tasks or no steps: empty curves, nothing to run
            return out
        if kvcache is None:
            kv = torch.empty(self.kv_numel(N, H), dtype=torch.float32, device=dev)
        else:
            kv = kvcache
            if not (kv.is_cuda and kv.dtype == torch.float32 and kv.is_contiguous()
                    and kv.numel() >= self.kv_numel(N, H)):
                raise ValueError(f"kvcache must be a contiguous fp32 device tensor of >= {self.kv_numel(N, H)} elements")
        u_d = None if uniforms is None else _dev(uniforms, torch.float64, dev)
        g_d = None if noise is None else _dev(noise, torch.float64, dev)
        args = _lib.BanditRolloutArgs(
            N, H, A, int(bandit_type), int(bool(sample)), 0, int(first_task), float(var), int(seed) & (2 ** 64 - 1),
            _p(means_d).value, None if u_d is None else _p(u_d).value, None if g_d is None else _p(g_d).value,
            _p(kv).value, _p(out["actions"]).value, _p(out["rewards"]).value, _p(out["arm_value"]).value,
            None if out["logits"] is None else _p(out["logits"]).value, int(counter) & (2 ** 64 - 1))
        _lib.call("dpt_rollout_bandit", self._h, ctypes.byref(args), _stream())
        out["_keep"] = (kv, means_d, u_d, g_d)
        return out

    def rollout_darkroom(self, goals, Heps, horizon, ctx_episodes, dim=10, perms=None, sample=True, temp=1.0,
                         seed=0, counter=0, first_task=0, uniforms=None, want_actions=False, want_logits=False,
                         want_forwards=False):
        """Fused DarkRoom online evaluation (evals/eval_darkroom.py:20-84) on device.

        Returns dict of device tensors: returns (N, Heps) int32, actions (N, Heps*horizon)
        int32, logits (Heps*horizon, N, 5) f32 and forwards (N, Heps) int32 (window
        forwards run per task and episode: one per distinct state per episode under
        set_darkroom_memo) if requested.  Raises
        NotImplementedError outside sd=2 / A=5 / window <= darkroom_max_window() (use the
        per-step path).
        """
        dev = device()
        goals_d = _dev(goals, torch.int32, dev).contiguous()
        N = goals_d.shape[0]
        steps = int(Heps) * int(horizon)
        perms_d = None if perms is None else _dev(perms, torch.int32, dev).contiguous()
        u_d = None if uniforms is None else _dev(uniforms, torch.float64, dev).contiguous()
        out = dict(returns=torch.empty((N, int(Heps)), dtype=torch.int32, device=dev))
        out["actions"] = torch.empty((N, steps), dtype=torch.int32, device=dev) if want_actions else None
        out["logits"] = torch.empty((steps, N, 5), dtype=torch.float32, device=dev) if want_logits else None
        out["forwards"] = torch.empty((N, int(Heps)), dtype=torch.int32, device=dev) if want_forwards else None
        if N == 0 or steps == 0:  # no tasks or no steps: empty returns, nothing to run
            for k in ("returns", "forwards"):
                if out[k] is not None:
                    out[k].zero_()
            return out
        n_ws = ctypes.c_int64()
        _lib.call("dpt_darkroom_workspace_numel_window", N, 1 + int(ctx_episodes) * int(horizon), ctypes.byref(n_ws))
        ws = torch.empty(n_ws.value, dtype=torch.float32, device=dev) if _darkroom_ws else None
        args = _lib.DarkroomRolloutArgs(
            N, int(Heps), int(horizon), int(ctx_episodes), int(dim), int(bool(sample)), int(first_task),
            int(seed) & (2 ** 64 - 1), int(counter), float(temp), 0, _p(goals_d).value,
            None if perms_d is None else _p(perms_d).value, None if u_d is None else _p(u_d).value,
            _p(out["returns"]).value, None if out["actions"] is None else _p(out["actions"]).value,
            None if out["logits"] is None else _p(out["logits"]).value,
            None if out["forwards"] is None else _p(out["forwards"]).value,
            None if ws is None else _p(ws).value)
        _lib.call("dpt_rollout_darkroom", self._h, ctypes.byref(args), _stream())
        out["_keep"] = (goals_d, perms_d, u_d, ws)
        return out


# ----------------------------------------------------------------------------- element-wise ops

def select_action(logits, sample, temp=1.0, uniforms=None, seed=0, counter=0, first_task=0):
    logits = _dev(logits, torch.float32)
    N, A = logits.shape
    u = None if uniforms is None else _dev(uniforms, torch.float64, logits.device)
    out = torch.empty(N, dtype=torch.int32, device=logits.device)
    _lib.call("dpt_select_action", _p(logits), N, A, int(bool(sample)), float(temp), _p(u), int(seed),
              int(counter), int(first_task), _p(out), _stream())
    return out


def bandit_step(means, action, var, bandit_type=BANDIT_GAUSSIAN, noise=None, seed=0, counter=0,
                first_task=0):
    means = _dev(means, torch.float64)
    N, A = means.shape
    a = _dev(action, torch.int32, means.device)
    g = None if noise is None else _dev(noise, torch.float64, means.device)
    r = torch.empty(N, dtype=torch.float64, device=means.device)
    v = torch.empty(N, dtype=torch.float64, device=means.device)
    _lib.call("dpt_bandit_step", _p(means), N, A, _p(a), int(bandit_type), float(var), _p(g), int(seed),
              int(counter), int(first_task), _p(r), _p(v), _stream())
    return r, v


def darkroom_step(state, action, goal, perm=None, dim=10):
    s = _dev(state, torch.int32)
    N = s.shape[0]
    a = _dev(action, torch.int32, s.device)
    g = _dev(goal, torch.int32, s.device)
    pm = None if perm is None else _dev(perm, torch.int32, s.device)
    ns = torch.empty_like(s)
    r = torch.empty(N, dtype=torch.int32, device=s.device)
    _lib.call("dpt_darkroom_step", _p(s), _p(a), _p(g), _p(pm), N, int(dim), _p(ns), _p(r), _stream())
    return ns, r


def darkroom_opt_action(state, goal, perm=None):
    s = _dev(state, torch.int32)
    g = _dev(goal, torch.int32, s.device)
    pm = None if perm is None else _dev(perm, torch.int32, s.device)
    out = torch.empty(s.shape[0], dtype=torch.int32, device=s.device)
    _lib.call("dpt_darkroom_opt_action", _p(s), _p(g), _p(pm), s.shape[0], _p(out), _stream())
    return out


def draw(kind, seed, counter, first_task, N, stream_id):
    """The Philox draws the kernels use (kind 0 uniform, 1 normal) -> (N,) float64 device tensor."""
    out = torch.empty(int(N), dtype=torch.float64, device=device())
    _lib.call("dpt_draw", int(kind), int(seed), int(counter), int(first_task), int(N), int(stream_id),
              _p(out), _stream())
    return out


# ----------------------------------------------------------------------------- data generation

def rollin_bandit(means, probs, H, var, bandit_type=BANDIT_GAUSSIAN, uniforms=None, noise=None, seed=0,
                  first_task=0):
    """collect_data.py:23-53 for all tasks at once -> (actions (N,H) int32, rewards (N,H) f64) on device."""
    means = _dev(means, torch.float64)
    N, A = means.shape
    probs = _dev(probs, torch.float64, means.device)
    u = None if uniforms is None else _dev(uniforms, torch.float64, means.device)
    g = None if noise is None else _dev(noise, torch.float64, means.device)
    acts = torch.empty((N, int(H)), dtype=torch.int32, device=means.device)
    rews = torch.empty((N, int(H)), dtype=torch.float64, device=means.device)
    _lib.call("dpt_rollin_bandit", _p(means), _p(probs), N, A, int(H), int(bandit_type), float(var), _p(u), _p(g),
              int(seed), int(first_task), _p(acts), _p(rews), _stream())
    return acts, rews


def rollin_darkroom(goals, H, dim=10, perm=None, mode=0, states=None, actions=None, seed=0, first_task=0):
    """collect_data.py:83-111 (+ query / expert label, :199-201) for all tasks at once (device tensors)."""
    goals = _dev(goals, torch.int32)
    N = goals.shape[0]
    dev = goals.device
    pm = None if perm is None else _dev(perm, torch.int32, dev)
    si = None if states is None else _dev(states, torch.int32, dev)
    ai = None if actions is None else _dev(actions, torch.int32, dev)
    out = dict(states=torch.empty((N, int(H), 2), dtype=torch.int32, device=dev),
               actions=torch.empty((N, int(H)), dtype=torch.int32, device=dev),
               next_states=torch.empty((N, int(H), 2), dtype=torch.int32, device=dev),
               rewards=torch.empty((N, int(H)), dtype=torch.int32, device=dev),
               query=torch.empty((N, 2), dtype=torch.int32, device=dev),
               opt_action=torch.empty(N, dtype=torch.int32, device=dev))
    _lib.call("dpt_rollin_darkroom", _p(goals), _p(pm), N, int(H), int(dim), int(mode), _p(si), _p(ai), int(seed),
              int(first_task), _p(out["states"]), _p(out["actions"]), _p(out["next_states"]), _p(out["rewards"]),
              _p(out["query"]), _p(out["opt_action"]), _stream())
    return out


# ----------------------------------------------------------------------------- classical baselines

from ._lib import (POLICY_EMP, POLICY_LCB, POLICY_LINUCB, POLICY_OPT, POLICY_THOMPSON,  # noqa: E402,F401
                   POLICY_UCB)


def rollout_policy(policy, means, H, var, bandit_type=BANDIT_GAUSSIAN, online=True, sample=True, c=1.0,
                   ts_std=0.1, ts_prior_mean=0.5, ts_prior_var=1 / 12.0, arms=None, seed=0, first_task=0,
                   noise=None, policy_noise=None, ctx_actions=None, ctx_rewards=None, counter=0):
    """Fused classical-policy rollout (dpt_rollout_policy); optional prefix context (N, C).
    ``counter``: the Philox step counter of step 0 (step h draws at counter + h)."""
    dev = device()
    means_d = _dev(means, torch.float64, dev)
    N, A = means_d.shape
    H = int(H)
    C = 0 if ctx_actions is None else int(np.asarray(ctx_actions).shape[1]) if not isinstance(
        ctx_actions, torch.Tensor) else int(ctx_actions.shape[1])
    keep = [means_d]

    def opt(x, dt):
        if x is None:
            return None
        t = _dev(x, dt, dev)
        keep.append(t)
        return _p(t).value

    if policy_noise is not None:
        # the kernel indexes the injected draws by the policy's own layout (dpt_policies.hip):
        # Thompson (H, N, A) when sampling, (H, 100, N, A) for the 100-draw vote; LinUCB (N,)
        # uniforms for an empty context's random arm; no other policy reads them
        got = int(policy_noise.numel() if isinstance(policy_noise, torch.Tensor) else np.asarray(policy_noise).size)
        if int(policy) == POLICY_THOMPSON:
            want = H * N * A if sample else H * 100 * N * A
            if got != want:
                raise ValueError(f"policy_noise has {got} draws; Thompson (sample={bool(sample)}) reads {want}")
        elif int(policy) == POLICY_LINUCB and got < N:  # only step 0's row (N,) is read
            raise ValueError(f"policy_noise has {got} draws; LinUCB reads the first {N}")
    n = ctypes.c_int64()
    _lib.call("dpt_policy_workspace_numel", N, A, C + H, ctypes.byref(n))  # 0: contexts live in LDS
    ws = torch.empty(max(n.value, 1), dtype=torch.float64, device=dev)
    out = dict(actions=torch.empty((N, H), dtype=torch.int32, device=dev),
               rewards=torch.empty((N, H), dtype=torch.float64, device=dev),
               arm_value=torch.empty((N, H), dtype=torch.float64, device=dev))
    d = 0 if arms is None else int(np.asarray(arms).shape[1])
    args = _lib.PolicyRolloutArgs(
        N, H, A, int(policy), int(bool(online)), int(bandit_type), int(bool(sample)), d, int(first_task), float(var),
        float(c), float(ts_std), float(ts_prior_mean), float(ts_prior_var), int(seed) & (2 ** 64 - 1),
        _p(means_d).value, opt(arms, torch.float64), opt(noise, torch.float64), opt(policy_noise, torch.float64),
        _p(ws).value, _p(out["actions"]).value, _p(out["rewards"]).value, _p(out["arm_value"]).value, C, int(counter),
        opt(ctx_actions, torch.int32), opt(ctx_rewards, torch.float64))
    _lib.call("dpt_rollout_policy", ctypes.byref(args), _stream())
    out["_keep"] = (keep, ws)
    return out


def regret_moments(arm_value, opt, mode=_lib.REGRET_SUMS, mean=None):
    """One pass of the device regret statistics (evals/eval_bandit.py:169-178, scipy's two-pass
    form): arm_value (N, H) fp64, opt (N,) fp64 -> (2, H) fp64 sums over tasks of
    (diff, cumsum(diff)) for REGRET_SUMS, or of their squared deviations from ``mean`` (2, H)
    for REGRET_CENTRED."""
    dev = device()
    av = _dev(arm_value, torch.float64, dev)
    op = _dev(opt, torch.float64, dev).reshape(-1)
    N, H = av.shape
    if op.shape[0] != N:
        raise ValueError(f"opt has {op.shape[0]} tasks, arm_value {N}")
    n = ctypes.c_int64()
    _lib.call("dpt_regret_workspace_numel", N, H, ctypes.byref(n))
    ws = torch.empty(n.value, dtype=torch.float64, device=dev)
    out = torch.empty((2, H), dtype=torch.float64, device=dev)
    mn = None if mean is None else _dev(mean, torch.float64, dev)
    _lib.call("dpt_regret_moments", _p(av), _p(op), N, H, int(mode), _p(mn), _p(ws), _p(out), _stream())
    return out


def regret_max_steps():
    n = ctypes.c_int32()
    _lib.call("dpt_regret_max_steps", ctypes.byref(n))
    return n.value


def set_decode_tile(tile):
    """Tasks per workgroup of the decode kernels (8: two workgroups per CU; 16: one)."""
    _lib.call("dpt_tuning_set", _lib.TUNE_DECODE_TILE, int(tile))


def set_cache_budget(nbytes):
    """Bytes of the Infinity Cache the bandit rollout may fill with its earliest positions' cached
    rows (default policy, resident across steps); 0 streams every row non-temporally.  Cache
    policy only: results are bit-identical for any value."""
    _lib.call("dpt_tuning_set", _lib.TUNE_CACHE_BUDGET, int(nbytes))


def set_block0_mfma(on):
    """Bandit rollout, 5 arms at tile 8: block 0's attention on the matrix cores, or one wave per
    task on the vector ALUs (default).  Same algebra; the fp32 summation order differs."""
    _lib.call("dpt_tuning_set", _lib.TUNE_BLOCK0_MFMA, int(bool(on)))


def set_select_fast(on):
    """select_action for 5 and 20 arms: the fp32 cdf with the exact fp64 cdf within 2^-15 of an edge
    (default), or the fp64 cdf for every sample.  Bit-identical either way."""
    _lib.call("dpt_tuning_set", _lib.TUNE_SELECT_FAST, int(bool(on)))


_darkroom_memo = True
_darkroom_ws = True


def darkroom_max_window():
    """Largest window (1 + R*horizon tokens) of the fused DarkRoom rollout: 512 with the per-task
    workspace (16 waves per task above 256 tokens), 256 without it."""
    return 512 if _darkroom_ws else 256


def set_darkroom_workspace(on):
    """DarkRoom rollout: keep the context tokens' layer-0 inputs and queries in a per-task device
    workspace for the episode (default) or recompute them every step (the workspace-free path)."""
    global _darkroom_ws
    _darkroom_ws = bool(on)


def set_darkroom_memo(on):
    """DarkRoom rollout: one window forward per distinct query state per episode (default) or per step.
    Applies to the fused kernel and to the per-step device loop (evals/eval_darkroom.py)."""
    global _darkroom_memo
    _lib.call("dpt_tuning_set", _lib.TUNE_DARKROOM_MEMO, int(bool(on)))
    _darkroom_memo = bool(on)


def darkroom_memo():
    return _darkroom_memo


def set_prefill(on):
    """Windows up to DeviceModel.prefill_max_window() as one MFMA prefill (default) or position by position."""
    _lib.call("dpt_tuning_set", _lib.TUNE_PREFILL, int(bool(on)))
