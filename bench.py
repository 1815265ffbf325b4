"""Headline benchmark: env-steps/sec with the DPT policy in the loop, 5-arm bandit, H=500.

One "step" = one full online rollout (evals/eval_bandit.py:56-103 with the DPT
controller sampling, ctrls/ctrl_bandit.py:422-444) of N_local = 4096 tasks x
H = 500 env steps on each GPU (BASELINE.json configs[1]; weak scaling over
GPUs, tasks sharded by global id, Philox keyed by global task id), followed by
the RCCL all-gather of the per-task arm-value curves (the regret inputs).
Inputs (weights, means) are resident in HBM before the timed region.

Prints ONE JSON line on rank 0.  Launch: python bench.py [--gpus N --steps K --warmup W]
(multi-GPU: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def synthetic_state_dict(n_layer, state_dim, action_dim, horizon, seed=0):
    """GPT-2 init scheme (N(0,0.02); c_proj N(0, 0.02/sqrt(2L)); LN 1/0; biases 0) for the
    reference Transformer (models/net.py:25-39) + a seeded 0.05*N(0,1) perturbation."""
    from models.net import Transformer
    cfg = dict(horizon=horizon, state_dim=state_dim, action_dim=action_dim, n_layer=n_layer, n_embd=32,
               n_head=1, dropout=0.0, test=True)
    torch.manual_seed(seed)
    m = Transformer(cfg)
    rs = np.random.RandomState(seed)
    sd = {}
    for k, v in m.state_dict().items():
        if k.endswith("wte.weight"):
            continue
        sd[k] = v + 0.05 * torch.from_numpy(rs.standard_normal(tuple(v.shape)).astype(np.float32))
    return sd


def algorithmic_bytes(N, H, n_layer, E=32):
    """Minimal HBM bytes of one fused rollout launch: at step h the K/V rows of
    positions < h are streamed (2*L*E*4 B each), the new K/V row is written,
    and means[a] (8 B) is read + action (4 B), reward and arm value (8 B each)
    are written."""
    kvb = 2 * n_layer * E * 4
    per_task = kvb * H * (H - 1) // 2 + (kvb + 28) * H
    return N * per_task


def cpu_baseline(sd, means, H, var, n_layer, A):
    from oracle import c_oracle
    import dpt_hip
    threads = max(1, min(16, os.cpu_count() or 1))
    blob = dpt_hip.pack_weights(sd, n_layer).numpy()
    npos = 4 * (1 + H)
    rs = np.random.RandomState(7)
    n_rec = 128  # ~10-20 s of CPU work on a 16-thread share
    u = rs.uniform(size=(H, n_rec))
    g = rs.normal(size=(H, n_rec))
    t0 = time.perf_counter()
    c_oracle.bandit_rollout(blob, n_layer, A, npos, means[:n_rec], H, var, u, g, True, True, threads)
    t_rec = time.perf_counter() - t0
    n_kv = 2048
    u = rs.uniform(size=(H, n_kv))
    g = rs.normal(size=(H, n_kv))
    t0 = time.perf_counter()
    c_oracle.bandit_rollout(blob, n_layer, A, npos, means[:n_kv], H, var, u, g, True, False, threads)
    t_kv = time.perf_counter() - t0
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return ({"value": n_rec * H / t_rec, "unit": "env-steps/s", "cores": threads, "kind": "port",
             "sample": f"{n_rec} tasks x H={H} full online rollout, reference algorithm (whole window "
                       f"re-forwarded every step, evals/eval_bandit.py:56-103), fp32 C + OpenMP, {cpu}",
             "seconds": t_rec},
            {"value": n_kv * H / t_kv, "unit": "env-steps/s", "cores": threads, "kind": "port-kvcache",
             "sample": f"{n_kv} tasks x H={H}, same C oracle with an exact K/V cache", "seconds": t_kv})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--tasks", type=int, default=4096, help="tasks per GPU")
    ap.add_argument("--H", type=int, default=500)
    ap.add_argument("--arms", type=int, default=5)
    ap.add_argument("--var", type=float, default=0.3)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import dpt_hip

    N, H, A, L = args.tasks, args.H, args.arms, args.layers
    sd = synthetic_state_dict(L, 1, A, H, seed=0)
    model = dpt_hip.DeviceModel(sd, L, 1, A, 4 * (1 + H))
    means_all = np.random.RandomState(1).uniform(0, 1, (N * world, A))
    first = rank * N
    means = torch.from_numpy(means_all[first:first + N]).cuda()
    gather = torch.empty((world * N, H), dtype=torch.float64, device="cuda") if world > 1 else None

    def one(step_idx):
        out = model.rollout_bandit(means, H, args.var, True, seed=1000 + step_idx, first_task=first)
        if dist is not None:
            dist.all_gather_into_tensor(gather, out["arm_value"])
        return out

    for w in range(args.warmup):
        one(w)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        out = model.rollout_bandit(means, H, args.var, True, seed=2000 + k, first_task=first)
        ev[k][1].record()
        if dist is not None:
            dist.all_gather_into_tensor(gather, out["arm_value"])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        km = torch.tensor([kern_ms], dtype=torch.float64, device="cuda")
        dist.all_reduce(km, op=dist.ReduceOp.MAX)
        kern_ms = float(km.item())

    env_steps = world * N * H * args.steps
    value = env_steps / elapsed
    abytes = algorithmic_bytes(N, H, L)
    achieved = abytes / (kern_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_rollout_bandit.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    line = {
        "metric": "env-steps/sec/GPU (DPT policy in loop), 5-arm bandit H=500, 1/2/4/8 MI355X",
        "value": value,
        "unit": "env-steps/s (whole job, all GPUs)",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (model) / f64 (env, rewards)",
        "data": "synthetic: seeded GPT-2-init weights (+0.05 N(0,1)), means ~ RandomState(1).U(0,1)",
        "config": {"workload": f"{A}-arm Gaussian bandit online eval, DPT sampling policy in the loop, "
                               f"H={H}, {N} tasks/GPU, var={args.var}, L={L} E=32 1 head",
                   "tasks_per_gpu": N, "horizon": H, "arms": A, "parallelism": f"task-sharded x{world}",
                   "env_steps_per_step": world * N * H},
        "per_gpu_value": value / world,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "rollout_bandit_kernel", "kernel_ms": kern_ms,
                     "algorithmic_bytes_per_launch": abytes},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base, kv = cpu_baseline(sd, means_all, H, args.var, L, A)
        line["cpu_baseline"] = base
        line["cpu_baseline_kvcache"] = kv
    if rank == 0:
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
