"""The multi-rank device path on the GPU box (one GPU, so the ranks share it over gloo; the
measured 8-GPU runs use RCCL, bench.py): the fused HIP rollouts of every rank's task block, the
device branch of regret_stats_allreduce under an initialised process group, gather_rows, and
bench.py launched by torch.distributed.run.  Ranks are spawned processes (spawn context: they
start fresh interpreters, nothing is forked from a GPU-initialised process)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bandit_case(n_total, H):
    import bench
    sd, _ = bench.synthetic_state_dict(4, 1, 5, H)
    means = np.random.RandomState(11).uniform(0, 1, (n_total, 5))
    return sd, means


def _darkroom_case(n_total):
    import bench
    sd, _ = bench.synthetic_state_dict(4, 2, 5, 100)
    goals = np.array([(j, i) for j in range(10) for i in range(10)])
    np.random.RandomState(0).shuffle(goals)
    return sd, goals[np.arange(n_total) % 100]


def _worker(rank, port, n_bandit, H, n_dark, q):
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import dpt_hip
    from dpt_hip.distributed import gather_rows, regret_stats_allreduce, shard
    # bandit: the fused rollout of this rank's block, statistics over all tasks (device branch)
    sd, means = _bandit_case(n_bandit, H)
    first, count = shard(n_bandit, WORLD, rank)
    m = dpt_hip.DeviceModel(sd, 4, 1, 5, 4 * (1 + H))
    local = torch.from_numpy(means[first:first + count]).cuda()
    out = m.rollout_bandit(local, H, 0.3, True, seed=555, first_task=first)
    stats = regret_stats_allreduce(local.max(dim=1, keepdim=True).values, out["arm_value"], n_bandit)
    curves = gather_rows(out["arm_value"], n_bandit)
    # darkroom: the fused online eval of this rank's block, returns gathered
    sdd, goals = _darkroom_case(n_dark)
    f2, c2 = shard(n_dark, WORLD, rank)
    md = dpt_hip.DeviceModel(sdd, 4, 2, 5, 404)
    rd = md.rollout_darkroom(goals[f2:f2 + c2], 6, 100, 1, seed=777, first_task=f2)
    rets = gather_rows(rd["returns"], n_dark)
    if rank == 0:
        q.put({"stats": {k: v.cpu().numpy() for k, v in stats.items()}, "curves": curves.cpu().numpy(),
               "returns": rets.cpu().numpy()})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(600)
def test_two_ranks_on_device_equal_one_process():
    """2 ranks x (uneven) task blocks: the gathered bandit curves and DarkRoom returns equal one
    process's bit for bit (Philox keyed by the global task id); the regret mean / SEM curves from
    the device moments and two all_reduces equal the single-process device statistics to fp64
    summation order (evals/eval_bandit.py:169-178)."""
    import dpt_hip
    from dpt_hip.distributed import regret_stats_allreduce
    n_bandit, H, n_dark = 1003, 200, 301
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, n_bandit, H, n_dark, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = q.get(timeout=540)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sd, means = _bandit_case(n_bandit, H)
    m = dpt_hip.DeviceModel(sd, 4, 1, 5, 4 * (1 + H))
    md_means = torch.from_numpy(means).cuda()
    out = m.rollout_bandit(md_means, H, 0.3, True, seed=555)
    assert np.array_equal(got["curves"], out["arm_value"].cpu().numpy())
    single = regret_stats_allreduce(md_means.max(dim=1, keepdim=True).values, out["arm_value"], n_bandit)
    for k, v in single.items():
        np.testing.assert_allclose(got["stats"][k], v.cpu().numpy(), rtol=1e-12, atol=1e-14)
    sdd, goals = _darkroom_case(n_dark)
    md = dpt_hip.DeviceModel(sdd, 4, 2, 5, 404)
    rd = md.rollout_darkroom(goals, 6, 100, 1, seed=777)
    assert np.array_equal(got["returns"], rd["returns"].cpu().numpy())


@pytest.mark.timeout(600)
def test_bench_under_torchrun_two_ranks():
    """bench.py --gpus 2 launched by torch.distributed.run (gloo: both ranks on this box's one GPU):
    one JSON line from rank 0 with n_gpus 2, the per-GPU workload unchanged and the whole-job
    env-step count of both ranks, in the headline and in the config-5 / config-4 sub-objects."""
    env = dict(os.environ, DPT_BENCH_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--tasks", "512", "--H", "100"]
    res = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=500)
    assert res.returncode == 0, res.stderr[-3000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-3000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert line["config"]["tasks_per_gpu"] == 512 and line["config"]["horizon"] == 100
    assert line["config"]["env_steps_per_step"] == 2 * 512 * 100
    assert line["value"] > 0 and line["roofline"]["kernel_ms"] > 0
    # the config-5 and config-4 sub-objects: every rank's shard, whole-job env steps of both ranks
    assert line["darkroom_c5_shard"]["config"]["env_steps_per_step"] == 2 * 8192 * 40 * 100
    assert line["linear_c4_shard"]["config"]["env_steps_per_step"] == 2 * 4096 * 1000
    assert line["linear_c4_shard"]["value"] > 0 and line["darkroom_c5_shard"]["value"] > 0


def _worker_nccl(port, n_bandit, H, q):
    sys.path[:0] = [PKG, ROOT]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    import dpt_hip
    from dpt_hip.distributed import gather_rows, regret_stats_allreduce
    sd, means = _bandit_case(n_bandit, H)
    m = dpt_hip.DeviceModel(sd, 4, 1, 5, 4 * (1 + H))
    local = torch.from_numpy(means).cuda()
    out = m.rollout_bandit(local, H, 0.3, True, seed=555)
    stats = regret_stats_allreduce(local.max(dim=1, keepdim=True).values, out["arm_value"], n_bandit)
    curves = gather_rows(out["arm_value"], n_bandit)
    t = torch.tensor([1.5, 2.5], dtype=torch.float64, device="cuda")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing reduction
    dist.barrier()
    q.put({"stats": {k: v.cpu().numpy() for k, v in stats.items()}, "curves": curves.cpu().numpy(),
           "t": t.cpu().numpy()})
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_rccl_backend_paths_single_rank():
    """The RCCL ("nccl" backend) branches the 8-GPU run takes, exercised with one rank on this box's
    GPU: init_process_group("nccl", device_id=...), the device-tensor all_reduce of
    regret_stats_allreduce, all_gather_into_tensor in gather_rows, bench.py's MAX reduction.
    Results equal the process-local computation."""
    import dpt_hip
    from dpt_hip.distributed import regret_stats_allreduce
    n_bandit, H = 777, 120
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker_nccl, args=(_free_port(), n_bandit, H, q))
    p.start()
    got = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    sd, means = _bandit_case(n_bandit, H)
    m = dpt_hip.DeviceModel(sd, 4, 1, 5, 4 * (1 + H))
    md_means = torch.from_numpy(means).cuda()
    out = m.rollout_bandit(md_means, H, 0.3, True, seed=555)
    assert np.array_equal(got["curves"], out["arm_value"].cpu().numpy())
    single = regret_stats_allreduce(md_means.max(dim=1, keepdim=True).values, out["arm_value"], n_bandit)
    for k, v in single.items():
        assert np.array_equal(got["stats"][k], v.cpu().numpy()), k
    assert np.array_equal(got["t"], [1.5, 2.5])
