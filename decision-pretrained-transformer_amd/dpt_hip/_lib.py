"""ctypes binding of libdpt_hip.so (include/dpt_hip.h).

The library is built in-tree (``make -C csrc`` / ``__graft_entry__.build()``)
and loaded from this directory.  There is no fallback: a missing or stale
library raises ImportError/OSError at first use, so nothing silently runs on
the CPU.  Return codes are mapped to the reference's Python exceptions
(envs/bandit_env.py:16,63,67-68; envs/darkroom_env.py:39,58-59).
"""
import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# DPT_HIP_LIB: another build's file name in this directory (A/B runs of kernel variants)
LIB_PATH = os.path.join(_HERE, os.environ.get("DPT_HIP_LIB", "libdpt_hip.so"))
ABI_VERSION = 7

DPT_OK = 0
DPT_EINVAL = -1
DPT_EEPISODE_ENDED = -2
DPT_EHIP = -3
DPT_ENOMEM = -4
DPT_EUNSUPPORTED = -5

BANDIT_GAUSSIAN = 0
BANDIT_BERNOULLI = 1
BANDIT_F32 = 16
STREAM_SELECT = 0
STREAM_REWARD = 1
STREAM_ROLLIN = 2
STREAM_DROPOUT = 3  # training dropout masks (dpt_train_desc)
STREAM_POLICY = 16  # + arm index (baseline-policy draws)

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float
_f64 = ctypes.c_double


class ModelDesc(ctypes.Structure):
    _fields_ = [("n_layer", _i32), ("n_embd", _i32), ("state_dim", _i32), ("action_dim", _i32),
                ("n_positions", _i32), ("reserved", _i32 * 3)]


class BanditRolloutArgs(ctypes.Structure):
    _fields_ = [("N", _i32), ("H", _i32), ("A", _i32), ("type", _i32), ("sample", _i32),
                ("reserved0", _i32), ("first_task", _i64), ("var", _f64), ("seed", _u64),
                ("means", _c_void_p), ("uniforms", _c_void_p), ("noise", _c_void_p),
                ("kvcache", _c_void_p), ("actions_out", _c_void_p), ("rewards_out", _c_void_p),
                ("arm_value_out", _c_void_p), ("logits_out", _c_void_p), ("counter", _u64)]


# name -> (restype, argtypes); mirrors include/dpt_hip.h exactly
SIGNATURES = {
    "dpt_abi_version": (_i32, []),
    "dpt_last_error": (ctypes.c_char_p, []),
    "dpt_device_count": (_i32, [ctypes.POINTER(_i32)]),
    "dpt_weights_numel": (_i32, [ctypes.POINTER(ModelDesc), ctypes.POINTER(_i64)]),
    "dpt_model_create": (_i32, [ctypes.POINTER(ModelDesc), _c_void_p, ctypes.POINTER(_c_void_p)]),
    "dpt_model_free": (_i32, [_c_void_p]),
    "dpt_forward_window": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                  _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p]),
    "dpt_kvcache_numel": (_i32, [_c_void_p, _i32, _i32, ctypes.POINTER(_i64)]),
    "dpt_decode_step": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p]),
    "dpt_select_action": (_i32, [_c_void_p, _i32, _i32, _i32, _f32, _c_void_p, _u64, _u64, _i64,
                                 _c_void_p, _c_void_p]),
    "dpt_bandit_step": (_i32, [_c_void_p, _i32, _i32, _c_void_p, _i32, _f64, _c_void_p, _u64, _u64, _i64,
                               _c_void_p, _c_void_p, _c_void_p]),
    "dpt_darkroom_step": (_i32, [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _c_void_p,
                                 _c_void_p, _c_void_p]),
    "dpt_darkroom_opt_action": (_i32, [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p]),
    "dpt_draw": (_i32, [_i32, _u64, _u64, _i64, _i32, _u32, _c_void_p, _c_void_p]),
    "dpt_rollout_bandit": (_i32, [_c_void_p, ctypes.POINTER(BanditRolloutArgs), _c_void_p]),
    "dpt_rollin_bandit": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _f64, _c_void_p, _c_void_p, _u64,
                                 _i64, _c_void_p, _c_void_p, _c_void_p]),
    "dpt_rollin_darkroom": (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _i32, _c_void_p, _c_void_p, _u64, _i64,
                                   _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p]),
}

_lock = threading.Lock()
_lib = None


def load():
    """Load and type the library once; raises if it is missing or the ABI differs."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built (run `make -C csrc` or __graft_entry__.build()); "
                              "the DPT hot path has no CPU fallback")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # (tests/test_abi.py requires every header symbol; an older build loaded for an A/B may
            # lack newer entry points, which then fail when called)
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        v = lib.dpt_abi_version()
        if v != ABI_VERSION:
            raise ImportError(f"libdpt_hip ABI {v} != bindings ABI {ABI_VERSION}")
        _lib = lib
        return lib


class EpisodeEndedError(ValueError):
    pass


def check(rc):
    """Map a DPT_E* code to the reference's exception types."""
    if rc == DPT_OK:
        return
    msg = load().dpt_last_error().decode(errors="replace")
    if rc == DPT_EEPISODE_ENDED:
        raise EpisodeEndedError("Episode has already ended")
    if rc == DPT_EINVAL:
        raise ValueError(msg)
    if rc == DPT_EUNSUPPORTED:
        raise NotImplementedError(msg)
    if rc == DPT_ENOMEM:
        raise MemoryError(msg)
    raise RuntimeError(msg)


def call(name, *args):
    check(getattr(load(), name)(*args))


POLICY_OPT, POLICY_EMP, POLICY_UCB, POLICY_THOMPSON, POLICY_LCB, POLICY_LINUCB = range(6)


class PolicyRolloutArgs(ctypes.Structure):
    _fields_ = [("N", _i32), ("H", _i32), ("A", _i32), ("policy", _i32), ("online", _i32), ("type", _i32),
                ("sample", _i32), ("lin_d", _i32), ("first_task", _i64), ("var", _f64), ("c", _f64),
                ("ts_std", _f64), ("ts_prior_mean", _f64), ("ts_prior_var", _f64), ("seed", _u64),
                ("means", _c_void_p), ("arms", _c_void_p), ("noise", _c_void_p), ("policy_noise", _c_void_p),
                ("workspace", _c_void_p), ("actions_out", _c_void_p), ("rewards_out", _c_void_p),
                ("arm_value_out", _c_void_p), ("C", _i32), ("step0", _i32), ("ctx_actions", _c_void_p),
                ("ctx_rewards", _c_void_p)]


SIGNATURES.update({
    "dpt_policy_workspace_numel": (_i32, [_i32, _i32, _i32, ctypes.POINTER(_i64)]),
    "dpt_rollout_policy": (_i32, [ctypes.POINTER(PolicyRolloutArgs), _c_void_p]),
})

TUNE_DECODE_TILE = 1
TUNE_PREFILL = 2
TUNE_DARKROOM_MEMO = 3
TUNE_CACHE_BUDGET = 4
TUNE_BLOCK0_MFMA = 5
TUNE_SELECT_FAST = 6
TUNE_POLICY_WAVE = 7
SIGNATURES["dpt_tuning_set"] = (_i32, [_i32, _i64])


class DarkroomRolloutArgs(ctypes.Structure):
    _fields_ = [("N", _i32), ("Heps", _i32), ("horizon", _i32), ("ctx_episodes", _i32), ("dim", _i32),
                ("sample", _i32), ("first_task", _i64), ("seed", _u64), ("counter", _u64), ("temp", _f32),
                ("reserved0", _i32), ("goals", _c_void_p), ("perms", _c_void_p), ("uniforms", _c_void_p),
                ("returns_out", _c_void_p), ("actions_out", _c_void_p), ("logits_out", _c_void_p),
                ("forwards_out", _c_void_p), ("workspace", _c_void_p)]


SIGNATURES["dpt_prefill_max_window"] = (_i32, [_c_void_p, ctypes.POINTER(_i32)])
SIGNATURES["dpt_rollout_darkroom"] = (_i32, [_c_void_p, ctypes.POINTER(DarkroomRolloutArgs), _c_void_p])

REGRET_SUMS = 0
REGRET_CENTRED = 1
SIGNATURES["dpt_regret_max_steps"] = (_i32, [ctypes.POINTER(_i32)])
SIGNATURES["dpt_regret_workspace_numel"] = (_i32, [_i32, _i32, ctypes.POINTER(_i64)])
SIGNATURES["dpt_regret_moments"] = (_i32, [_c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p,
                                           _c_void_p, _c_void_p])
SIGNATURES["dpt_darkroom_workspace_numel"] = (_i32, [_i32, ctypes.POINTER(_i64)])
SIGNATURES["dpt_darkroom_workspace_numel_window"] = (_i32, [_i32, _i32, ctypes.POINTER(_i64)])


class TrainDesc(ctypes.Structure):
    _fields_ = [("n_layer", _i32), ("n_embd", _i32), ("state_dim", _i32), ("action_dim", _i32),
                ("n_positions", _i32), ("batch", _i32), ("window", _i32), ("reserved", _i32),
                ("dropout", ctypes.c_float), ("reserved2", _i32), ("dropout_seed", ctypes.c_uint64)]


TRAIN_FORWARD_ONLY = 1  # dpt_train_desc.reserved flag (DPT_TRAIN_FORWARD_ONLY)
TRAIN_LAST_ONLY = 2  # with it: preds at the last position only (DPT_TRAIN_LAST_ONLY)


SIGNATURES["dpt_train_blob_numel"] = (_i32, [ctypes.POINTER(TrainDesc), ctypes.POINTER(_i64)])
SIGNATURES["dpt_train_workspace_numel"] = (_i32, [ctypes.POINTER(TrainDesc), ctypes.POINTER(_i64)])
SIGNATURES["dpt_train_forward"] = (_i32, [ctypes.POINTER(TrainDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                          _c_void_p])
SIGNATURES["dpt_train_backward"] = (_i32, [ctypes.POINTER(TrainDesc), _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                                           _c_void_p, _c_void_p])
SIGNATURES["dpt_rollout_bandit_generic_workspace_numel"] = (_i32, [ctypes.POINTER(TrainDesc), _i32, _i32,
                                                                   ctypes.POINTER(_i64)])
SIGNATURES["dpt_rollout_bandit_generic"] = (_i32, [ctypes.POINTER(TrainDesc), _c_void_p,
                                                   ctypes.POINTER(BanditRolloutArgs), _c_void_p])
