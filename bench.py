"""Headline benchmark: env-steps/sec with the DPT policy in the loop, 5-arm bandit, H=500.

One "step" = one full online rollout (evals/eval_bandit.py:56-103 with the DPT
controller sampling, ctrls/ctrl_bandit.py:422-444) of N_local = 4096 tasks x
H = 500 env steps on each GPU (BASELINE.json configs[1]; weak scaling over
GPUs: contiguous task blocks, Philox keyed by global task id), followed by
the regret statistics over all tasks (evals/eval_bandit.py:169-178: mean and
SEM curves, from an RCCL all_reduce of per-step moments for N > 1).
Inputs (weights, means) are resident in HBM before the timed region.

Other workloads (not the headline line): --workload linear (config 4 shard:
20-arm linear bandit, H=1000, 4096 tasks/GPU), --workload darkroom (config 3:
DarkRoom 10x10, H=100, Heps=40, 4096 tasks/GPU).

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

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
FP32_MFMA_PEAK_TF = 157.3  # MI355X_MICROARCH.md: FP32 matrix 157.3 TFLOP/s (spec)
BF16_MFMA_PEAK_TF = 2500.0  # MI355X_MICROARCH.md: BF16 ~2.5 PFLOP/s dense
# fp32-accurate products on the fp16 matrix cores (dpt_mfma_fwd.h mfma_x3, fp16 two-part
# splits): one K=32 tile is three v_mfma_f32_16x16x32_f16 (16 cycles each) instead of eight
# v_mfma_f32_16x16x4_f32 (32 cycles each), so the fp32-equivalent ceiling of every product
# of the DarkRoom forward is 256/48 x the fp32 one
X3_PEAK_TF = FP32_MFMA_PEAK_TF * 256 / 48


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
    return sd, m


def algorithmic_bytes(N, H, n_layer, E=32):
    """Minimal HBM bytes of one fused rollout launch (rollout_bandit_kernel's
    algorithm): at step h, blocks 1..L-1 stream the cached LayerNorm output y_p
    of positions < h (E*4 B each; y serves as both key and value on folded
    weights) and block 0 reads the 16-B token record of each position
    < h (action, reward and the ln_1 mean / rstd: its attention is recomputed from
    the tokens); the new y rows and record are written, and means[a] (8 B) is
    read + action (4 B), reward and arm value (8 B each) are written.  wpe and the
    weights are shared by every task and served from L2 (not counted)."""
    per_pos = (n_layer - 1) * E * 4 + 16
    per_task = per_pos * H * (H - 1) // 2 + (per_pos + 28) * H
    return N * per_task


def kvcache_bytes(N, H, n_layer, E=32):
    """SURVEY.md 8(d)'s bytes for the plain K/V-cache decode (every block's K/V
    streamed, 2*L*E*4 B per position): what the same rollout would move without
    the block-0 recompute."""
    kvb = 2 * n_layer * E * 4
    return N * (kvb * H * (H - 1) // 2 + (kvb + 28) * H)


def window_flops(T, n_layer, F, A, E=32, folded=True, split=False):
    """FLOPs of one causal window forward over T tokens (embed, L blocks, ln_f, head):
    per block 2*T*E*(E + E + 4E + 4E) dense with the folded attention the kernels run
    (u = y G + g0 and (sum P y) Wvp; 3E + E for c_attn + c_proj unfolded)
    + 2 * 2*E * T(T+1)/2 attention.  split=True: (matrix products = dense + attention, the
    embedding and head) separately."""
    dense = 2 * T * E * ((E if folded else 3 * E) + E + 4 * E + 4 * E)
    attn = 2 * 2 * E * T * (T + 1) // 2
    if split:
        return n_layer * (dense + attn), 2 * T * F * E + 2 * E * A
    return n_layer * (dense + attn) + 2 * T * F * E + 2 * E * A


def cpu_info():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """The host cores this process may run on: the affinity mask, capped by a cgroup CPU quota
    (cgroup v2 cpu.max) when one is set; with nproc, the quota and the CPU model for the line."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    threads = max(1, min(aff, int(quota)) if quota else aff)
    return threads, {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
                     "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cpu_model": cpu_info()}


def cpu_baseline(sd, means, H, var, n_layer, A, n_rec=None, n_kv=2048):
    """The C oracle (oracle/dpt_oracle.c, fp32 as the reference's torch forward) on every host core
    this process may use: the reference algorithm (whole window re-forwarded each step) on a
    bounded sample of the workload, BASELINE config 1 (64 tasks, H=100, 5 arms) in full, and the
    same arithmetic with an exact K/V cache."""
    from oracle import c_oracle
    import dpt_hip
    threads, hw = host_cpus()
    n_rec = n_rec or 4 * max(16, threads)  # four tasks per thread (~6 s at H=500 on the GPU box's EPYC)
    blob = dpt_hip.pack_weights(sd, n_layer).numpy()
    npos = 4 * (1 + H)
    rs = np.random.RandomState(7)
    u, g = rs.uniform(size=(H, n_rec)), rs.normal(size=(H, n_rec))
    t0 = time.perf_counter()
    c_oracle.bandit_rollout(blob, n_layer, A, npos, means[:n_rec], H, var, u, g, True, True, threads)
    t_rec = time.perf_counter() - t0
    # config 1 in full: 64 tasks x H=100 (its own means, RandomState(1); the model's first wpe rows)
    H1, N1 = 100, 64
    m1 = np.random.RandomState(1).uniform(0, 1, (N1, A))
    u1, g1 = rs.uniform(size=(H1, N1)), rs.normal(size=(H1, N1))
    t0 = time.perf_counter()
    c_oracle.bandit_rollout(blob, n_layer, A, npos, m1, H1, var, u1, g1, True, True, threads)
    t_c1 = time.perf_counter() - t0
    u, g = rs.uniform(size=(H, n_kv)), rs.normal(size=(H, n_kv))
    t0 = time.perf_counter()
    c_oracle.bandit_rollout(blob, n_layer, A, npos, means[:n_kv], H, var, u, g, True, False, threads)
    t_kv = time.perf_counter() - t0
    return ({"value": n_rec * H / t_rec, "unit": "env-steps/s", "cores": threads, "kind": "port",
             "sample": f"{n_rec} tasks x H={H} full online rollout, reference algorithm (whole window "
                       f"re-forwarded every step, evals/eval_bandit.py:56-103), fp32 C + OpenMP",
             "seconds": t_rec, "host": hw,
             "config1_full": {"value": N1 * H1 / t_c1, "unit": "env-steps/s", "seconds": t_c1,
                              "sample": f"BASELINE config 1 in full: {N1} tasks x H={H1}, 5 arms, var {var}, "
                                        "reference algorithm"}},
            {"value": n_kv * H / t_kv, "unit": "env-steps/s", "cores": threads, "kind": "port-kvcache",
             "sample": f"{n_kv} tasks x H={H}, same C oracle with an exact K/V cache", "seconds": t_kv})


def cpu_baseline_darkroom(sd, goals, H, n_layer, n_tasks=None, n_eps=8):
    """DarkRoom online eval on the host cores: the float64 C restatement (oracle/dpt_oracle.c,
    pinned to the reference's rollouts) with the reference's algorithm -- one full window forward
    per env step, no memo (evals/eval_darkroom.py:53-66) -- on the first n_eps episodes of
    n_tasks tasks (episode 0 has an empty window, the others the full 1 + H tokens)."""
    from oracle import c_oracle
    import dpt_hip
    threads, hw = host_cpus()
    n_tasks = n_tasks or 4 * max(8, threads)
    blob = dpt_hip.pack_weights(sd, n_layer).numpy()
    u = np.random.RandomState(7).uniform(size=(n_eps * H, n_tasks))
    t0 = time.perf_counter()
    c_oracle.darkroom_rollout(blob, n_layer, 4 * (1 + H), goals[:n_tasks], n_eps, H, 1, u, True, memo=False,
                              threads=threads)
    t = time.perf_counter() - t0
    return {"value": n_tasks * n_eps * H / t, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "seconds": t, "host": hw,
            "sample": f"{n_tasks} tasks x {n_eps} episodes x {H} steps of the online eval (episode 0 empty "
                      f"window, then 1+{H} tokens), reference algorithm: a full window forward every step, "
                      "float64 C + OpenMP"}


def stream_ceiling(N, H, n_layer, pin_positions, kernel_ms):
    """The bandit rollout's read pattern alone (scripts/stream_probe.hip: every step's y rows of
    blocks 1..L-1 exactly as attend_one reads them, no compute), timed here on the same GPU as the
    headline: its time plus the token records' share at the same rate is the floor of the launch's
    reads on this layout; frac = that floor / the rollout's kernel time."""
    import ctypes
    co = os.path.join(ROOT, "scripts", "stream_probe.co")
    if not os.path.exists(co):
        return None
    nblk = n_layer - 1
    y = torch.zeros(nblk * N * H * 32, dtype=torch.float32, device="cuda")
    out = torch.zeros(1, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    mod, fn = ctypes.c_void_p(), ctypes.c_void_p()
    if hip.hipModuleLoad(ctypes.byref(mod), co.encode()) or \
            hip.hipModuleGetFunction(ctypes.byref(fn), mod, b"stream_probe"):
        return None
    args = [ctypes.c_void_p(y.data_ptr()), ctypes.c_int(N), ctypes.c_int(H), ctypes.c_int(pin_positions),
            ctypes.c_int(nblk), ctypes.c_void_p(out.data_ptr())]
    ptrs = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.pointer(a), ctypes.c_void_p) for a in args])
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        if hip.hipModuleLaunchKernel(fn, (N + 7) // 8, 1, 1, 512, 1, 1, 0, stream, ptrs, None):
            return None
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    hip.hipModuleUnload(mod)
    ms = min(ts)
    ybytes = nblk * 128 * N * H * (H - 1) // 2
    rec_ms = ms * (algorithmic_bytes(N, H, n_layer) - ybytes) / ybytes  # token records etc. at the probe's rate
    return {"probe_ms": ms, "probe_TBps": ybytes / ms / 1e9, "floor_ms": ms + rec_ms,
            "frac": (ms + rec_ms) / kernel_ms, "kernel": "scripts/stream_probe.hip (y reads only, same layout)",
            "note": "floor = probe time of the y stream + the remaining algorithmic bytes at the probe's rate; "
                    "frac = floor / rollout kernel_ms (1.0 = the launch reads at its layout's measured ceiling)"}


def run_timed(one, steps, warmup, dist, backend, kernel_only):
    """W untimed warmup steps, then K steps bracketed by a barrier + synchronize on both sides;
    returns (elapsed s max over ranks, kernel ms: the rollout launch alone when kernel_only else
    the whole step, max over ranks)."""
    for w in range(warmup):
        one(w)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    for k in range(steps):
        ev[k][0].record()
        one(100 + k, kev[k])
        ev[k][1].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in (kev if kernel_only else ev)]))
    if dist is not None:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    return elapsed, kern_ms


def darkroom_workload(L, H, Heps, N, first, count, n_total, dist, memo):
    """BASELINE config 3 (config 5's per-GPU shard for --tasks 8192): the DarkRoom online eval
    (evals/eval_darkroom.py:20-84, DPT sampling controller) over this rank's task block."""
    import dpt_hip
    from ctrls.ctrl_darkroom import DarkroomTransformerController
    from dpt_hip.distributed import gather_rows
    from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec
    from evals import eval_darkroom
    dpt_hip.set_darkroom_memo(memo)
    sd, tmodel = synthetic_state_dict(L, 2, 5, H, seed=0)
    tmodel.load_state_dict({**sd, "transformer.wte.weight": tmodel.transformer.wte.weight}, strict=True)
    tmodel.cuda().eval()  # as eval.py:152 does
    goals = np.array([(j, i) for j in range(10) for i in range(10)])
    np.random.RandomState(0).shuffle(goals)   # collect_data.py:408-409 order, cycled to N
    goals_all = goals[np.arange(n_total) % 100]
    envs = [DarkroomEnv(10, g, H) for g in goals_all[first:first + count]]
    vec = DarkroomEnvVec(envs, first_task=first)

    def one(step_idx, ev=None):
        np.random.seed(step_idx)
        ctrl = DarkroomTransformerController(tmodel, batch_size=count, sample=True)
        ret = eval_darkroom.deploy_online_vec(vec, ctrl, Heps, H, H)
        if dist is not None:  # the per-task returns of every rank (online regret all-gather)
            gather_rows(torch.from_numpy(ret).cuda(), n_total)
        return ret

    def roofline(kern_ms):
        # The kernel runs one window forward per distinct query state per episode (the
        # window is fixed within an episode): replay the first timed step
        # (same np seed -> same draws -> same trajectory) untimed to count the forwards
        # it ran, and price the roofline on those, not on one forward per env step.
        np.random.seed(100)
        ctrl = DarkroomTransformerController(tmodel, batch_size=count, sample=True)
        fw = eval_darkroom.rollout_fused(vec, ctrl, Heps, H, H, want_forwards=True)["forwards"]
        fw = fw.to(torch.int64).sum(0).cpu().numpy()  # (Heps,) forwards over all tasks
        F = 2 * 2 + 5 + 1
        ref_flops = count * H * (window_flops(1, L, F, 5, folded=False) +
                                 (Heps - 1) * window_flops(1 + H, L, F, 5, folded=False))
        flops = int(fw[0]) * window_flops(1, L, F, 5) + int(fw[1:].sum()) * window_flops(1 + H, L, F, 5)
        achieved = flops / (kern_ms * 1e-3) / 1e12
        # the ceiling of this mix: the blocks' products (mfma_x3 on the fp16 cores) at X3_PEAK_TF,
        # the embedding and head (VALU) at the fp32 peak
        parts = [window_flops(1, L, F, 5, split=True), window_flops(1 + H, L, F, 5, split=True)]
        dense = int(fw[0]) * parts[0][0] + int(fw[1:].sum()) * parts[1][0]
        peak = flops / (dense / X3_PEAK_TF + (flops - dense) / FP32_MFMA_PEAK_TF)
        traffic = None  # HBM bytes read per launch (rocprofv3 FETCH_SIZE x2, scripts/profile_darkroom.sh)
        issue = None  # the issue roofline from the same PMC pass (scripts/pmc_darkroom.py)
        pmc = os.path.join(ROOT, "profiles", "pmc_rollout_darkroom.json")
        if os.path.exists(pmc) and count == 4096 and H == 100:
            pj = json.load(open(pmc))
            traffic = pj.get("hbm_fetch_bytes_corrected")
            if "simd_valu_or_mfma_busy_frac" in pj:
                issue = {k: pj[k] for k in ("simd_valu_issue_frac", "mfma_pipe_busy_frac", "valu_mfma_coexec_frac",
                                            "simd_valu_or_mfma_busy_frac", "avg_waves_per_simd")}
                issue["note"] = ("fractions of SIMD cycles from the committed PMC pass of this kernel at this "
                                 "config (profiles/pmc_rollout_darkroom.json): VALU issue, MFMA pipe busy, both, "
                                 "either -- the kernel is issue-bound, so this, not the MFMA-only peak, is its "
                                 "binding roofline")
        return {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "issue": issue,
                "frac": achieved / peak, "traffic": traffic,
                "peak_fp32_mfma": FP32_MFMA_PEAK_TF, "frac_of_fp32_mfma": achieved / FP32_MFMA_PEAK_TF,
                "matrix_flops_per_launch": dense,
                "kernel": "rollout_darkroom_kernel (one launch = one whole online eval)",
                "kernel_ms": kern_ms, "algorithmic_flops_per_launch": flops,
                "window_forwards_per_launch": int(fw.sum()),
                "reference_flops_per_launch": ref_flops,
                "note": "flops = window forwards the kernel ran (one per distinct state per episode) x "
                        "FLOPs of that window with the folded attention; the reference runs one unfolded "
                        "forward per env step (reference_flops_per_launch). peak = the ceiling of this "
                        "FLOP mix: every product of the blocks (dense and attention) as fp32-accurate "
                        "fp16 two-part split products (three 16x16x32 f16 MFMAs per K=32 tile: "
                        "157.3 x 256/48 TFLOP/s), embedding and head at the fp32 peak (157.3)"}

    workload = f"DarkRoom 10x10 online eval, DPT sampling policy, H=horizon={H}, Heps={Heps}, {N} tasks/GPU"
    # rollout_darkroom_kernel: every matrix product as fp16 two-part splits on
    # v_mfma_f32_16x16x32_f16 (h*h + h*m + m*h, fp32 accumulation: about 2^-21 relative per
    # product); LayerNorm, softmax, gelu, embedding, head in fp32; selection cdf in fp32
    # (the exact fp64 cdf within 2^-15 of an edge, select_fast)
    dtype = ("f16x2-split MFMA products (fp32 accumulate, ~2^-21/product) + f32 VALU / "
             "f32 selection cdf (f64 within 2^-15 of an edge); int32 grid")
    return dict(one=one, roofline=roofline, env_steps=n_total * Heps * H, workload=workload, dtype=dtype,
                cfg={"tasks_per_gpu": N, "horizon": H, "episodes": Heps}, sd=sd, goals=goals_all)


def bandit_workload(wl, L, H, var, first, count, n_total, rank):
    """BASELINE config 2 (wl "bandit": 5 arms, H=500, means ~ U(0,1)) or config 4's per-GPU shard
    (wl "linear": 20 arms, H=1000, collect_data.py:230-231 arms, theta ~ N(0,1)/sqrt(2)): the
    online eval (evals/eval_bandit.py:56-103 / eval_linear_bandit.py:54-97, DPT sampling
    controller) over this rank's task block, then the regret mean / SEM curves over all tasks."""
    import dpt_hip
    from dpt_hip.distributed import regret_stats_allreduce
    A, H = (5, H or 500) if wl == "bandit" else (20, H or 1000)
    sd, _ = synthetic_state_dict(L, 1, A, H, seed=0)
    model = dpt_hip.DeviceModel(sd, L, 1, A, 4 * (1 + H))
    if wl == "bandit":
        means_all = np.random.RandomState(1).uniform(0, 1, (n_total, A))
    else:  # collect_data.py:230-231 arms; theta ~ N(0,1)/sqrt(d)
        arms = np.random.RandomState(1234).normal(size=(A, 2)) / np.sqrt(2)
        thetas = np.random.RandomState(2).normal(0, 1, (n_total, 2)) / np.sqrt(2)
        means_all = np.stack([arms @ t for t in thetas])
    means = torch.from_numpy(means_all[first:first + count]).cuda()
    opt = means.max(dim=1, keepdim=True).values  # the Opt controller's arm value (eval_bandit.py:123-128)

    def one(step_idx, ev=None):
        if ev is not None:
            ev[0].record()
        out = model.rollout_bandit(means, H, var, True, seed=1000 + step_idx, first_task=first)
        if ev is not None:  # the rollout kernel's own span (the roofline's launch duration)
            ev[1].record()
        # the eval's output: suboptimality / cumulative-regret mean and SEM curves over all tasks
        # (evals/eval_bandit.py:169-178), from two all_reduces of 2 x H fp64 moments (RCCL for N>1)
        return regret_stats_allreduce(opt, out["arm_value"], n_total)

    def roofline(kern_ms, with_stream_ceiling=False):
        # kern_ms: HIP events around the one rollout launch (draws + rollout_bandit_kernel) on the
        # current stream
        abytes = algorithmic_bytes(count, H, L)
        achieved = abytes / (kern_ms * 1e-3) / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", f"pmc_rollout_{'bandit' if wl == 'bandit' else 'linear'}.json")
        if os.path.exists(pmc):
            p = json.load(open(pmc))
            if p.get("algorithmic_bytes_per_launch") == abytes:
                traffic = p.get("hbm_bytes_per_launch")
        roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "kernel": "rollout_bandit_kernel",
                "kernel_ms": kern_ms, "algorithmic_bytes_per_launch": abytes,
                "kvcache_bytes_per_launch": kvcache_bytes(count, H, L)}
        if with_stream_ceiling:
            pin = ctypes_pin_positions(count, H, L)
            sc = stream_ceiling(count, H, L, pin, kern_ms) if pin is not None else None
            if sc is not None:
                roof["stream_ceiling"] = sc
        return roof

    workload = (f"{A}-arm {'Gaussian' if wl == 'bandit' else 'linear (d=2)'} bandit online eval, DPT sampling "
                f"policy in the loop, H={H}, {count} tasks/GPU, var={var}, L={L} E=32 1 head")
    # rollout_bandit_kernel: fp32 VALU + v_mfma_f32_16x16x4_f32 products; env arithmetic fp64
    dtype = "f32 (model: VALU + f32 MFMA) / f64 (env, rewards)"
    return dict(one=one, roofline=roofline, env_steps=n_total * H, workload=workload, dtype=dtype,
                cfg={"tasks_per_gpu": count, "horizon": H, "arms": A}, sd=sd, means_all=means_all, H=H, A=A)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=("bandit", "linear", "darkroom"), default="bandit")
    ap.add_argument("--tasks", type=int, default=4096, help="tasks per GPU")
    ap.add_argument("--H", type=int, default=None)
    ap.add_argument("--var", type=float, default=0.3)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-darkroom", action="store_true",
                    help="bandit: skip the DarkRoom sub-object (darkroom_c3 / darkroom_c5_shard)")
    ap.add_argument("--no-linear", action="store_true",
                    help="bandit: skip the linear_c4_shard sub-object (BASELINE config 4's per-GPU shard)")
    ap.add_argument("--darkroom-memo", type=int, choices=(0, 1), default=1,
                    help="darkroom: 1 = one window forward per distinct state per episode, 0 = one per step")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; DPT_BENCH_BACKEND=gloo (ranks may then share a GPU) rehearses the
    # multi-rank path on a one-GPU box -- the measured runs use RCCL ("nccl")
    backend = os.environ.get("DPT_BENCH_BACKEND", "nccl")
    dev = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    from dpt_hip.distributed import shard

    N, L, wl = args.tasks, args.layers, args.workload
    n_total = N * world
    first, count = shard(n_total, world, rank)
    if wl in ("bandit", "linear"):
        bw = bandit_workload(wl, L, args.H, args.var, first, count, n_total, rank)
        one, env_steps_per_step, workload, cfg, dtype = bw["one"], bw["env_steps"], bw["workload"], bw["cfg"], \
            bw["dtype"]
        sd, means_all, H, A = bw["sd"], bw["means_all"], bw["H"], bw["A"]
    else:
        H, Heps = args.H or 100, 40
        dw = darkroom_workload(L, H, Heps, N, first, count, n_total, dist, args.darkroom_memo)
        one, env_steps_per_step, workload, cfg, dtype = dw["one"], dw["env_steps"], dw["workload"], dw["cfg"], \
            dw["dtype"]

    elapsed, kern_ms = run_timed(one, args.steps, args.warmup, dist, backend, wl in ("bandit", "linear"))
    value = env_steps_per_step * args.steps / elapsed
    if wl in ("bandit", "linear"):
        roof = bw["roofline"](kern_ms, with_stream_ceiling=rank == 0)
    else:
        roof = dw["roofline"](kern_ms)
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
        "dtype": dtype,
        "data": "synthetic: seeded GPT-2-init weights (+0.05 N(0,1)); tasks per SURVEY.md §8(d)",
        "config": dict(workload=workload, parallelism=f"task-sharded x{world}",
                       env_steps_per_step=env_steps_per_step, **cfg),
        "per_gpu_value": value / world,
        "roofline": roof,
    }
    if wl != "bandit":
        line["metric"] = f"env-steps/sec ({wl} workload; headline metric is --workload bandit)"
    if rank == 0 and world == 1 and wl == "bandit" and not args.no_cpu_baseline:
        base, kv = cpu_baseline(sd, means_all, H, args.var, L, A)
        line["cpu_baseline"] = base
        line["cpu_baseline_kvcache"] = kv
    if rank == 0 and world == 1 and wl == "darkroom" and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline_darkroom(dw["sd"], dw["goals"], H, L)
    if wl == "bandit" and not args.no_darkroom:
        # BASELINE config 3 (one GPU: 4096 tasks) or, on more GPUs, config 5's per-GPU shard (8192
        # tasks per GPU: config 5 itself at 8 GPUs), on the driver's clock beside the headline
        n_dr = 4096 if world == 1 else 8192
        f_dr, c_dr = shard(n_dr * world, world, rank)
        dw = darkroom_workload(L, 100, 40, n_dr, f_dr, c_dr, n_dr * world, dist, 1)
        dr_steps, dr_warm = 2, 1
        el, km = run_timed(dw["one"], dr_steps, dr_warm, dist, backend, False)
        sub = {"metric": "env-steps/sec (DarkRoom online eval, DPT policy in loop)",
               "value": dw["env_steps"] * dr_steps / el, "unit": "env-steps/s (whole job, all GPUs)",
               "steps": dr_steps, "warmup": dr_warm, "ms_per_step": el / dr_steps * 1e3, "dtype": dw["dtype"],
               "config": dict(workload=dw["workload"], env_steps_per_step=dw["env_steps"], **dw["cfg"]),
               "roofline": dw["roofline"](km)}
        if rank == 0 and world == 1 and not args.no_cpu_baseline:
            sub["cpu_baseline"] = cpu_baseline_darkroom(dw["sd"], dw["goals"], 100, L)
        line["darkroom_c3" if world == 1 else "darkroom_c5_shard"] = sub
        if world == 1:
            # config 5's per-GPU shard on one GPU: rank 0's 8192 of the 65,536 tasks (goals of the
            # global ids, Philox keyed by the global task id), one timed step
            dw = darkroom_workload(L, 100, 40, 8192, 0, 8192, 65536, None, 1)
            c5_steps = 1
            el, km = run_timed(dw["one"], c5_steps, 1, None, backend, False)
            env5 = 8192 * 40 * 100
            line["darkroom_c5_shard"] = {
                "metric": "env-steps/sec (DarkRoom online eval, DPT policy in loop)",
                "value": env5 * c5_steps / el, "unit": "env-steps/s (one GPU's shard)", "steps": c5_steps,
                "warmup": 1, "ms_per_step": el / c5_steps * 1e3, "dtype": dw["dtype"],
                "config": {"workload": dw["workload"].replace("65536 tasks/GPU", "8192 tasks/GPU") +
                           " (rank 0 of BASELINE config 5: 65,536 tasks over 8 GPUs)",
                           "env_steps_per_step": env5, "tasks_per_gpu": 8192, "horizon": 100, "episodes": 40},
                "roofline": dw["roofline"](km)}
    if wl == "bandit" and not args.no_linear:
        # BASELINE config 4 (20-arm linear, H=1000, 32,768 tasks over 8 GPUs): its 4096-task per-GPU
        # shard on every rank (config 4 itself at 8 GPUs), two timed steps
        f_l, c_l = shard(4096 * world, world, rank)
        lw = bandit_workload("linear", L, None, args.var, f_l, c_l, 4096 * world, rank)
        lin_steps = 2
        el, km = run_timed(lw["one"], lin_steps, 1, dist, backend, True)
        line["linear_c4_shard" if world < 8 else "linear_c4"] = {
            "metric": "env-steps/sec (20-arm linear bandit online eval, DPT policy in loop)",
            "value": lw["env_steps"] * lin_steps / el, "unit": "env-steps/s (whole job, all GPUs)",
            "steps": lin_steps, "warmup": 1, "ms_per_step": el / lin_steps * 1e3, "dtype": lw["dtype"],
            "config": dict(workload=lw["workload"] + " (BASELINE config 4: 32,768 tasks over 8 GPUs)",
                           env_steps_per_step=lw["env_steps"], **lw["cfg"]),
            "roofline": lw["roofline"](km)}
    if rank == 0:
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


def ctypes_pin_positions(N, H, n_layer, budget=224 << 20, chunk=64):
    """The Infinity-Cache residency of the rollout launch at the default budget (rollout_pin,
    dpt_decode.hip: whole 64-position stream chunks split over blocks 1..L-1), for the stream
    probe: the first pin positions are read with the default cache policy."""
    nb = n_layer - 1
    row = N * 32 * 4
    if nb <= 0:
        return None
    return int(min((budget // (row * chunk)) // nb * chunk, H))


if __name__ == "__main__":
    main()
