"""Bandit rollout (config 2) time vs the Infinity-Cache residency budget (DPT_TUNE_CACHE_BUDGET):
median of interleaved rounds per budget, HIP events around the launch."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

N, H = int(os.environ.get("SW_N", "4096")), int(os.environ.get("SW_H", "500"))
mibs = [int(x) for x in os.environ.get("SW_MIB", "128,192,208,224,240,252").split(",")]
sd, _ = bench.synthetic_state_dict(4, 1, 5, H)
m = dpt_hip.DeviceModel(sd, 4, 1, 5, 4 * (1 + H))
means = torch.from_numpy(np.random.RandomState(1).uniform(0, 1, (N, 5))).cuda()
m.rollout_bandit(means, H, 0.3, True, seed=0)
res = {b: [] for b in mibs}
for rnd in range(int(os.environ.get("SW_ROUNDS", "3"))):
    for b in mibs:
        dpt_hip.set_cache_budget(b << 20)
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.rollout_bandit(means, H, 0.3, True, seed=1 + rnd)
        e.record()
        torch.cuda.synchronize()
        res[b].append(a.elapsed_time(e))
        print(json.dumps({"round": rnd, "mib": b, "ms": res[b][-1]}), flush=True)
print(json.dumps({"median_ms": {b: float(np.median(v)) for b, v in res.items()}}))
