"""Evidence run (GPU): DarkRoom parity over the WHOLE population of BASELINE config 3 (4096 tasks)
and of config 5's first shard (8192 tasks), not a sample: the fused rollout against the float64 C
oracle fed the same Philox draws, with the acceptance rule of tests/test_gpu_kernels.py
(check_darkroom_tasks: each task compared up to its first differing action, which must fall on a
near-tie draw; logits within 1e-5 at every compared step; per-episode returns exactly).  The
oracle runs in chunks of 512 tasks with a progress line each.  Prints one JSON line per case.

    python scripts/dr_full_population.py > gpurun_out/dr_full_population.jsonl
    python scripts/dr_full_population.py --long       (windows 201 / 301 and the workspace-free dim 12)
    python scripts/dr_full_population.py --variants   (config 3 greedy, and with permuted actions)
    python scripts/dr_full_population.py --lastshard  (config 5's last shard)
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]

import bench  # noqa: E402
import dpt_hip  # noqa: E402
import philox_np  # noqa: E402
from oracle import c_oracle  # noqa: E402
from test_gpu_kernels import compared_steps, darkroom_config  # noqa: E402

LOGIT_TOL = 1e-5
CHUNK = 512


def case(label, N, seed, ctr, first_task, goals, R=1, dim=10, Heps=40, sample=True, perms=None):
    horizon, L = 100, 4
    steps = Heps * horizon
    sd, _ = bench.synthetic_state_dict(L, 2, 5, R * horizon)
    m = dpt_hip.DeviceModel(sd, L, 2, 5, 4 * (1 + R * horizon))
    out = m.rollout_darkroom(goals, Heps, horizon, R, dim=dim, perms=perms, sample=sample, seed=seed, counter=ctr,
                             first_task=first_task, want_actions=True, want_logits=True)
    lg_all = out["logits"].cpu().numpy()
    acts_all = out["actions"].cpu().numpy()
    rets_all = out["returns"].cpu().numpy()
    blob = dpt_hip.pack_weights(sd, L).numpy()
    n_all, err_max, ret_bad, t0 = [], 0.0, 0, time.time()
    for lo in range(0, N, CHUNK):
        tasks = np.arange(lo, min(N, lo + CHUNK))
        u = np.stack([philox_np.uniform(seed, ctr + k, first_task + tasks, dpt_hip.STREAM_SELECT)
                      for k in range(steps)]) if sample else None
        ref = c_oracle.darkroom_rollout(blob, L, 4 * (1 + R * horizon), goals[tasks], Heps, horizon, R, u, sample,
                                        perms=None if perms is None else perms[tasks], dim=dim,
                                        threads=bench.host_cpus()[0], want_logits=True)
        n = compared_steps(acts_all[tasks], ref["actions"], ref["margin"])
        for j, t in enumerate(tasks):
            k = min(n[j] + 1, steps)
            got, want = lg_all[:k, t].astype(np.float64), ref["logits"][:k, j]
            err_max = max(err_max, float((np.abs(got - want) / np.maximum(1.0, np.abs(want))).max()))
            ret_bad += int(not np.array_equal(rets_all[t, :n[j] // horizon], ref["returns"][j, :n[j] // horizon]))
        n_all.append(n)
        print(f"{label}: tasks {lo}..{tasks[-1]} done, {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
    n = np.concatenate(n_all)
    res = {"case": label, "tasks": int(N), "steps_per_task": steps, "window": 1 + R * horizon, "dim": dim,
           "task_steps_compared_frac": float(n.sum()) / (N * steps),
           "tasks_identical_all_steps_frac": float((n == steps).mean()),
           "tasks_with_a_near_tie_flip": int((n < steps).sum()),
           "max_scaled_logit_err": err_max, "logit_tol": LOGIT_TOL,
           "tasks_with_return_mismatch_before_flip": ret_bad,
           "pass": bool(err_max <= LOGIT_TOL and ret_bad == 0 and float(n.sum()) / (N * steps) >= 0.9)}
    print(json.dumps(res), flush=True)
    return res["pass"]


def main():
    if "--lastshard" in sys.argv:  # config 5's last rank (global tasks 57344..65535)
        ok = case("C5_shard7_all_8192", 8192, 1234, 0, 57344, darkroom_config(65536)[57344:])
    elif "--variants" in sys.argv:
        # config 3's population greedy (argmax: no draw, so every step must agree) and with a random
        # action permutation per task (the reference's permuted DarkRoom), sampled
        from oracle import dpt_oracle
        perms = dpt_oracle.perm_table()[np.random.RandomState(6).randint(0, 120, 4096)].astype(np.int32)
        ok = case("C3_greedy_all_4096", 4096, 0, 0, 0, darkroom_config(4096), sample=False)
        ok &= case("C3_permuted_all_4096", 4096, 11, 0, 0, darkroom_config(4096), perms=perms)
    elif "--long" in sys.argv:
        # the reference's longer contexts (H = 200 / 300 with horizon 100: windows 201 / 301), and the
        # workspace-free kernels (dim 12: 144 cells, no per-state table), on every task of smaller batches
        goals12 = np.random.RandomState(5).randint(0, 12, (1024, 2))
        ok = case("window201_all_1024", 1024, 7, 0, 0, darkroom_config(1024), R=2, Heps=20)
        ok &= case("window301_all_512", 512, 8, 0, 0, darkroom_config(512), R=3, Heps=12)
        ok &= case("dim12_window201_all_1024", 1024, 9, 0, 0, goals12, R=2, dim=12, Heps=20)
    else:
        ok = case("C3_all_4096", 4096, 99, 3, 0, darkroom_config(4096))
        ok &= case("C5_shard0_all_8192", 8192, 1234, 0, 0, darkroom_config(65536)[:8192])
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
