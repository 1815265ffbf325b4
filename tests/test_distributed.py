"""Multi-rank task sharding on CPU (gloo, world_size 2): a sharded online rollout gathered with
dpt_hip.distributed equals the unsharded run bit for bit (Philox keyed by global task id).
The per-rank rollout here is the C oracle fed numpy-Philox draws (test infrastructure);
on the GPU it is the fused HIP kernel (bench.py, test_gpu_kernels sharding test)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT, golden

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rollout_fn(blob, H, seed):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import philox_np
    from oracle import c_oracle

    def fn(means, first):
        n = means.shape[0]
        tasks = np.arange(first, first + n)
        u = np.stack([philox_np.uniform(seed, h, tasks, 0) for h in range(H)])
        g = np.stack([philox_np.normal(seed, h, tasks, 1) for h in range(H)])
        o = c_oracle.bandit_rollout(blob, 4, 5, 2004, means, H, 0.3, u, g, True, False, 1)
        return {"arm_value": torch.from_numpy(o["arm_value"]), "actions": torch.from_numpy(o["actions"])}
    return fn


def _worker(rank, port, blob, means, H, seed, q):
    import sys
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from dpt_hip.distributed import regret_stats_allreduce, shard, sharded_online
    full, local = sharded_online(_rollout_fn(blob, H, seed), means)
    first, count = shard(means.shape[0], WORLD, rank)
    opt = torch.from_numpy(np.repeat(means[first:first + count].max(1, keepdims=True), H, axis=1))
    stats = regret_stats_allreduce(opt, local["arm_value"], means.shape[0])
    if rank == 0:
        q.put(full.numpy())
        q.put({k: v.numpy() for k, v in stats.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_shard_blocks():
    from dpt_hip.distributed import shard
    for n in (1, 7, 64, 4097):
        for w in (1, 2, 3, 8):
            blocks = [shard(n, w, r) for r in range(w)]
            assert sum(c for _, c in blocks) == n
            assert all(blocks[r][0] + blocks[r][1] == blocks[r + 1][0] for r in range(w - 1))


@pytest.mark.timeout(300)
def test_gloo_world2_sharded_equals_single():
    import dpt_hip
    g = golden("forward_bandit5.npz")
    w = {k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w/")}
    blob = dpt_hip.pack_weights(w, 4).numpy()
    N, H, seed = 13, 10, 77  # uneven split 7 + 6
    means = np.random.RandomState(4).uniform(0, 1, (N, 5))
    single = _rollout_fn(blob, H, seed)(means, 0)["arm_value"].numpy()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, blob, means, H, seed, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    full = q.get(timeout=240)
    stats = q.get(timeout=60)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert np.array_equal(full, single)
    # online regret statistics through one all_reduce == the oracle's curves over all tasks
    import sys
    sys.path.insert(0, ROOT)
    from oracle import dpt_oracle as O
    opt = np.repeat(means.max(1, keepdims=True), H, axis=1)
    ref = O.regret_curves(opt, single)
    for k, v in ref.items():
        assert np.allclose(stats[k], v, rtol=1e-9, atol=1e-12), k


def _stats_worker(rank, port, opt, lnr, q):
    import sys
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    from dpt_hip.distributed import regret_stats_allreduce, shard
    first, count = shard(opt.shape[0], WORLD, rank)
    sl = slice(first, first + count)
    stats = regret_stats_allreduce(torch.from_numpy(opt[sl]), torch.from_numpy(lnr[sl]), opt.shape[0])
    if rank == 0:
        q.put({k: v.numpy() for k, v in stats.items()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_rank_without_tasks():
    """n_total=1 over 2 ranks: rank 1 owns no task (shard() gives it count 0) and still joins
    both all_reduces, so the job finishes and rank 0 gets the one task's curves."""
    rs = np.random.RandomState(2)
    H = 12
    opt = np.repeat(rs.uniform(0.5, 1.0, (1, 1)), H, axis=1)
    lnr = opt - rs.uniform(0, 0.5, (1, H))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, port, opt, lnr, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    stats = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    diff = (opt - lnr)[0]
    assert np.array_equal(stats["subopt_mean"], diff)
    assert np.allclose(stats["regret_mean"], np.cumsum(diff), rtol=1e-15, atol=0)


@pytest.mark.timeout(300)
def test_gloo_world2_regret_sem_matches_scipy():
    """regret_stats_allreduce at H=1000 (the linear-bandit horizon) on curves whose cumulative
    regret has a large mean relative to its spread: mean and SEM equal scipy.stats.sem over the
    gathered curves (evals/eval_bandit.py:169-178) to fp64 summation order."""
    import scipy.stats
    rs = np.random.RandomState(6)
    N, H = 301, 1000
    opt = np.repeat(rs.uniform(0.9, 1.0, (N, 1)), H, axis=1)
    lnr = opt - 0.25 - 1e-6 * rs.standard_normal((N, H))  # regret ~0.25 per step, tiny spread
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stats_worker, args=(r, port, opt, lnr, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    stats = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    diff = opt - lnr
    cr = np.cumsum(diff, axis=1)
    for key, x in (("subopt", diff), ("regret", cr)):
        assert np.allclose(stats[f"{key}_mean"], x.mean(0), rtol=1e-12, atol=0), key
        ref_sem = scipy.stats.sem(x, axis=0)
        assert np.allclose(stats[f"{key}_sem"], ref_sem, rtol=1e-6, atol=0), key
