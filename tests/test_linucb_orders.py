"""LinUCB's numpy arithmetic restated in OpenBLAS's rounding orders (csrc/dpt_linucb.h, shared with the
policy kernels) against numpy itself, on the host: the header is compiled with g++ into a small
harness, and every case is checked against the reference's own expressions
(ctrls/ctrl_bandit.py:503-526: cov = I + X^T X, np.linalg.inv, theta = cov_inv @ X^T @ r, value =
theta @ arm + c sqrt(arm @ cov_inv @ arm)).

Bit-exactness is relative to the BLAS numpy loads on this host, the one the reference fixtures were
recorded on (OpenBLAS picks its kernels per CPU at run time, so another host's numpy may round
differently): for every lin_d the kernel accepts (2..8) the inverse and every arm value must be
identical, over contexts that cross the syrk K-blocking (384 / 768 rows) and dgemv_t's 2048-row
blocks.  The GPU tests run the same header on the device against the recorded fixtures."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "decision-pretrained-transformer_amd", "csrc")

HARNESS = r"""
#include "dpt_linucb.h"
extern "C" int hc_linucb(const int* act, const double* rew, int n, const double* arms, int A, int d, double c,
                         double* values, double* ci) {
    return dpt::linucb_choose([&](int k) { return act[k]; }, [&](int k) { return rew[k]; }, n, arms, A, d, c,
                              values, ci);
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("linucb")
    src = d / "hc.cpp"
    src.write_text(HARNESS)
    so = d / "libhc.so"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared", f"-I{CSRC}",
                    str(src), "-o", str(so)], check=True)
    lib = ctypes.CDLL(str(so))
    P = ctypes.POINTER(ctypes.c_double)
    lib.hc_linucb.restype = ctypes.c_int
    lib.hc_linucb.argtypes = [ctypes.POINTER(ctypes.c_int), P, ctypes.c_int, P, ctypes.c_int, ctypes.c_int,
                              ctypes.c_double, P, P]
    return lib


def reference(arms, act, rew, c):
    """ctrls/ctrl_bandit.py:503-526, as written there (rewards (n, 1), as the batch holds them)"""
    d = arms.shape[1]
    actions_arms = arms[act]
    cov = 1.0 * np.eye(d) + actions_arms.T @ actions_arms
    cov_inv = np.linalg.inv(cov)
    theta = (cov_inv @ actions_arms.T @ rew[:, None]).flatten()
    vals = np.array([theta @ arm + c * np.sqrt(arm @ cov_inv @ arm) for arm in arms])
    return cov_inv, vals


def run(lib, arms, act, rew, c):
    A, d = arms.shape
    vals = np.zeros(A)
    ci = np.zeros((d, d))
    arms = np.ascontiguousarray(arms)
    act32 = np.ascontiguousarray(act, dtype=np.int32)
    rew = np.ascontiguousarray(rew)
    P = ctypes.POINTER(ctypes.c_double)
    best = lib.hc_linucb(act32.ctypes.data_as(ctypes.POINTER(ctypes.c_int)), rew.ctypes.data_as(P), len(act),
                         arms.ctypes.data_as(P), A, d, c, vals.ctypes.data_as(P), ci.ctypes.data_as(P))
    return best, ci, vals


def cases(d, count, seed):
    rng = np.random.RandomState(seed)
    for _ in range(count):
        A = rng.randint(2, 21)
        arms = rng.normal(0, 1, (A, d)) / np.sqrt(d)  # envs/bandit_env.py sample_linear's arm scale
        n = int(rng.choice([1, 2, 3, 4, 7, 50, 383, 500, 769, 900, 2051]))
        act = rng.randint(0, A, n)
        rew = rng.normal(0, 1, n)
        yield arms, act, rew


@pytest.mark.parametrize("d", [2, 3, 4, 5, 6, 7, 8])
def test_linucb_orders_bit_exact(harness, d):
    for arms, act, rew in cases(d, 100, d):
        ci_ref, v_ref = reference(arms, act, rew, 1.0)
        best, ci, vals = run(harness, arms, act, rew, 1.0)
        assert np.array_equal(ci, ci_ref), (d, len(act))
        assert np.array_equal(vals, v_ref), (d, len(act), vals - v_ref)
        assert best == int(np.argmax(v_ref))  # np.argmax is the first max, as the reference's '>' scan
