"""ctypes loader for oracle/build/libdpt_oracle.so (test / CPU-baseline infrastructure only)."""
import ctypes
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "build", "libdpt_oracle.so")
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
