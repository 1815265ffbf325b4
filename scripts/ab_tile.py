"""Interleaved in-process A/B of the decode tile (cdna guide §5.4 rule 24): N rounds x {16, 8}."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

H = int(os.environ.get("AB_H", "500"))
N = int(os.environ.get("AB_N", "4096"))
A = int(os.environ.get("AB_A", "5"))
sd, _ = bench.synthetic_state_dict(4, 1, A, H)
m = dpt_hip.DeviceModel(sd, 4, 1, A, 4 * (1 + H))
means = torch.from_numpy(np.random.RandomState(1).uniform(0, 1, (N, A))).cuda()
res = {16: [], 8: []}
for rnd in range(int(os.environ.get("AB_ROUNDS", "4"))):
    for tile in (16, 8):
        dpt_hip.set_decode_tile(tile)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.rollout_bandit(means, H, 0.3, True, seed=rnd)
        b.record()
        torch.cuda.synchronize()
        if rnd > 0:
            res[tile].append(a.elapsed_time(b))
abytes = bench.algorithmic_bytes(N, H, 4)
print(json.dumps({str(t): {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
                           "TBps": abytes / (np.median(v) * 1e-3) / 1e12} for t, v in res.items()}))
