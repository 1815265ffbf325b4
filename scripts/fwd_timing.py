"""Transformer.forward (dpt_forward_window) timing: MFMA prefill vs the
position-by-position K/V path, at the DarkRoom window (T = 101) and a bandit
offline context; prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


res = {}
for name, sd, A, H, N, C in (("darkroom_C3", 2, 5, 100, 4096, 100), ("bandit_offline_T128", 1, 5, 500, 200, 127),
                             ("bandit_offline_T501", 1, 5, 500, 200, 500), ("bandit_T501_N4096", 1, 5, 500, 4096, 500)):
    sdict, _ = bench.synthetic_state_dict(4, sd, A, H, seed=0)
    m = dpt_hip.DeviceModel(sdict, 4, sd, A, 4 * (1 + H))
    rs = np.random.RandomState(0)
    dev = dpt_hip.device()
    q = torch.from_numpy(rs.randint(0, 10, (N, sd)).astype(np.float32)).to(dev)
    cs = torch.from_numpy(rs.randint(0, 10, (N, C, sd)).astype(np.float32)).to(dev)
    cn = torch.from_numpy(rs.randint(0, 10, (N, C, sd)).astype(np.float32)).to(dev)
    ca = torch.from_numpy(np.eye(A, dtype=np.float32)[rs.randint(0, A, (N, C))]).to(dev)
    cr = torch.from_numpy(rs.rand(N, C).astype(np.float32)).to(dev)
    row = {"N": N, "T": C + 1}
    for on in (True, False):
        dpt_hip.set_prefill(on)
        ms = timed(lambda: m.forward_window(q, cs, ca, cn, cr, out_mode=0))
        row["prefill_ms" if on else "positionwise_ms"] = ms
    dpt_hip.set_prefill(True)
    flops = N * bench.window_flops(C + 1, 4, 2 * sd + A + 1, A)
    row["prefill_tflops"] = flops / (row["prefill_ms"] * 1e-3) / 1e12
    row["speedup"] = row["positionwise_ms"] / row["prefill_ms"]
    res[name] = row
print(json.dumps(res))
