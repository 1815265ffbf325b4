"""numpy Philox4x32-10 with the counter/key convention of csrc/dpt_common.h (test helper)."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)


def philox(seed, step, task, stream):
    task = np.asarray(task, dtype=np.int64).astype(np.uint64)
    step = np.uint64(step)
    c0 = np.full(task.shape, step & MASK, dtype=np.uint64)
    c1 = task & MASK
    c2 = np.full(task.shape, np.uint64(stream), dtype=np.uint64)
    c3 = (task >> np.uint64(32)) ^ (step >> np.uint64(32))
    k0 = np.uint64(int(seed) & 0xFFFFFFFF)
    k1 = np.uint64((int(seed) >> 32) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & MASK, lo1, (hi0 ^ c3 ^ k1) & MASK, lo0
        k0 = (k0 + np.uint64(W0)) & MASK
        k1 = (k1 + np.uint64(W1)) & MASK
    return c0, c1, c2, c3


def u53(a, b):
    return ((a >> np.uint64(5)).astype(np.float64) * 67108864.0
            + (b >> np.uint64(6)).astype(np.float64)) * (1.0 / 9007199254740992.0)


def uniform(seed, step, task, stream):
    x = philox(seed, step, task, stream)
    return u53(x[0], x[1])


def normal(seed, step, task, stream):
    x = philox(seed, step, task, stream)
    u1 = 1.0 - u53(x[0], x[1])
    u2 = u53(x[2], x[3])
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def dropout_keep(seed, p, site, shape):
    """The training kernels' dropout factors of one site (include/dpt_hip.h dpt_train_desc):
    element e kept iff word e % 4 of Philox(seed, (site, e / 4, DPT_STREAM_DROPOUT = 3)) >=
    ceil(p 2^32) (p as float32), kept elements times float32(1 / (1 - p)); float64 array."""
    p32 = np.float32(p)
    thr = min(int(np.ceil(np.float64(p32) * 2.0 ** 32)), 2 ** 32 - 1)
    scale = np.float64(np.float32(1.0) / (np.float32(1.0) - p32))
    n = int(np.prod(shape))
    w = np.stack(philox(seed, site, np.arange((n + 3) // 4), 3), 1).reshape(-1)[:n]
    return np.where(w >= np.uint64(thr), scale, 0.0).reshape(shape)
