"""ctypes loader for oracle/build/libdpt_oracle.so (test / CPU-baseline infrastructure only)."""
import ctypes
import os

import numpy as np

# DPT_ORACLE_LIB selects another build of the same source (make -C oracle asan: the
# AddressSanitizer / UBSan build that tests/test_oracle_sanitized.py runs the checks on)
_LIB = os.environ.get("DPT_ORACLE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "build",
                                                        "libdpt_oracle.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        _lib.dpt_oracle_bandit_rollout.restype = ctypes.c_int
        _lib.dpt_oracle_bandit_rollout.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_int,
                                                   ctypes.c_int, ctypes.c_double, P, P, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_int, P, P, P, P]
    return _lib


def bandit_rollout(blob, L, A, npos, means, H, var, u, g, sample=True, recompute=True, threads=1,
                   want_logits=False):
    """Same contract as dpt_oracle.bandit_online_rollout (fp32, packed dpt_hip.h blob)."""
    blob = np.ascontiguousarray(blob, np.float32)
    means = np.ascontiguousarray(means, np.float64)
    N = means.shape[0]
    u = np.ascontiguousarray(u if u is not None else np.zeros((H, N)), np.float64)
    g = np.ascontiguousarray(g, np.float64)
    acts = np.zeros((N, H), np.int32)
    rew = np.zeros((N, H))
    av = np.zeros((N, H))
    lg = np.zeros((H, N, A), np.float32) if want_logits else None
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = load().dpt_oracle_bandit_rollout(p(blob), L, A, npos, p(means), N, H, var, p(u), p(g), int(sample),
                                          int(recompute), int(threads), p(acts), p(rew), p(av), p(lg))
    if rc:
        raise ValueError("oracle rollout rejected the shape")
    return dict(actions=acts, rewards=rew, arm_value=av, cum_means=av.T, logits=lg)


def bandit_rollout_f64(blob, L, A, npos, means, H, var, u, g, sample=True, recompute=False, threads=1,
                       want_logits=False):
    """The bandit rollout with a float64 forward (dpt_oracle_bandit_rollout_f64): logits rounded
    to float32, then the reference's float32 softmax / float64 choice.  Also returns ``margin``
    (H, N): the distance of each step's uniform to the nearest interior cdf edge."""
    lib = load()
    if not hasattr(lib, "_bf64"):
        P = ctypes.c_void_p
        i = ctypes.c_int
        lib.dpt_oracle_bandit_rollout_f64.restype = i
        lib.dpt_oracle_bandit_rollout_f64.argtypes = [P, i, i, i, P, i, i, ctypes.c_double, P, P, i, i, i,
                                                      P, P, P, P, P]
        lib._bf64 = True
    blob = np.ascontiguousarray(blob, np.float32)
    means = np.ascontiguousarray(means, np.float64)
    N = means.shape[0]
    u = np.ascontiguousarray(u if u is not None else np.zeros((H, N)), np.float64)
    g = np.ascontiguousarray(g, np.float64)
    assert u.shape == (H, N) and g.shape == (H, N)
    acts = np.zeros((N, H), np.int32)
    rew = np.zeros((N, H))
    av = np.zeros((N, H))
    margin = np.zeros((H, N))
    lg = np.zeros((H, N, A), np.float32) if want_logits else None
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.dpt_oracle_bandit_rollout_f64(p(blob), L, A, npos, p(means), N, H, var, p(u), p(g), int(sample),
                                           int(recompute), int(threads), p(acts), p(rew), p(av), p(lg), p(margin))
    if rc:
        raise ValueError("oracle rollout rejected the shape")
    return dict(actions=acts, rewards=rew, arm_value=av, cum_means=av.T, logits=lg, margin=margin)


def darkroom_rollout(blob, L, npos, goals, Heps, horizon, R, u=None, sample=True, perms=None, dim=10, memo=True,
                     threads=1, want_logits=False):
    """Same contract as dpt_oracle.darkroom_online_rollout (float64 forward, packed dpt_hip.h
    blob); u (Heps*horizon, N) or None for greedy.  Also returns ``margin`` (steps, N): the
    distance of each step's uniform to the nearest interior cdf edge."""
    lib = load()
    if not hasattr(lib, "_dr"):
        P = ctypes.c_void_p
        i = ctypes.c_int
        lib.dpt_oracle_darkroom_rollout.restype = i
        lib.dpt_oracle_darkroom_rollout.argtypes = [P, i, i, P, P, i, i, i, i, i, P, i, i, i, P, P, P, P]
        lib._dr = True
    blob = np.ascontiguousarray(blob, np.float32)
    goals = np.ascontiguousarray(goals, np.int32)
    N = goals.shape[0]
    steps = Heps * horizon
    u = None if u is None else np.ascontiguousarray(np.asarray(u).reshape(steps, N), np.float64)
    perms = None if perms is None else np.ascontiguousarray(perms, np.int32)
    rets = np.zeros((N, Heps), np.int32)
    acts = np.zeros((N, steps), np.int32)
    margin = np.zeros((steps, N))
    lg = np.zeros((steps, N, 5), np.float32) if want_logits else None
    p = lambda a: None if a is None else a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    rc = lib.dpt_oracle_darkroom_rollout(p(blob), L, npos, p(goals), p(perms), N, Heps, horizon, R, dim, p(u),
                                         int(sample), int(memo), int(threads), p(rets), p(acts), p(lg), p(margin))
    if rc:
        raise ValueError("oracle darkroom rollout rejected the shape")
    return dict(returns=rets, actions=acts, logits=lg, margin=margin)
