"""Fit rollout time(H) = a*H + b*H^2: a = fixed per-step cost, b*H^2 = K/V streaming."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

N = int(os.environ.get("SW_N", "4096"))
Hs = [int(h) for h in os.environ.get("SW_H", "16,64,128,256,500").split(",")]
sd, _ = bench.synthetic_state_dict(4, 1, 5, 500)
m = dpt_hip.DeviceModel(sd, 4, 1, 5, 2004)
means = torch.from_numpy(np.random.RandomState(1).uniform(0, 1, (N, 5))).cuda()
out = {}
for tile in [int(t) for t in os.environ.get("SW_TILES", "16,8").split(",")]:
    dpt_hip.set_decode_tile(tile)
    ts = []
    for H in Hs:
        m.rollout_bandit(means, H, 0.3, True, seed=0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        m.rollout_bandit(means, H, 0.3, True, seed=1)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    X = np.stack([np.array(Hs, float), np.array(Hs, float) ** 2], 1)
    coef = np.linalg.lstsq(X, np.array(ts), rcond=None)[0]
    # marginal rate of the steps between consecutive horizons: algorithmic bytes / time
    by = [bench.algorithmic_bytes(N, H, 4) for H in Hs]
    marg = [(by[i + 1] - by[i]) / ((ts[i + 1] - ts[i]) * 1e-3) / 1e12 for i in range(len(Hs) - 1)]
    out[tile] = {"H": Hs, "ms": ts, "per_step_fixed_us": coef[0] * 1e3, "stream_ms_at_500": coef[1] * 500 ** 2,
                 "fixed_ms_at_500": coef[0] * 500, "marginal_TBps": marg}
print(json.dumps(out))
