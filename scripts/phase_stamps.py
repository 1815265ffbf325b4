"""Per-phase cycle shares of decode_position (diagnostic build libdpt_hip_stamps.so).
Phases: 0 embed+ln1 | 1 c_attn | 2 attention | 3 c_proj+ln2 | 4 c_fc->mlp | 5 reduce+ln | 6 head | 7 select+env."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
from dpt_hip import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__), "libdpt_hip_stamps.so")
lib = _lib.load()
lib.dpt_debug_stamps.restype = ctypes.c_int
lib.dpt_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

names = ["embed+ln1", "c_attn", "attention", "c_proj+ln2", "c_fc->mlp", "reduce+ln", "head", "select+env"]
sd, _ = bench.synthetic_state_dict(4, 1, 5, 500)
m = dpt_hip.DeviceModel(sd, 4, 1, 5, 2004)
N = int(os.environ.get("ST_N", "4096"))
means = torch.from_numpy(np.random.RandomState(1).uniform(0, 1, (N, 5))).cuda()
res = {}
for tile in [int(t) for t in os.environ.get("ST_TILES", "16,8").split(",")]:
    dpt_hip.set_decode_tile(tile)
    for H in [int(h) for h in os.environ.get("ST_H", "64,500").split(",")]:
        m.rollout_bandit(means, H, 0.3, True, seed=0)
        torch.cuda.synchronize()
        lib.dpt_debug_stamps(None, 0, 1)
        m.rollout_bandit(means, H, 0.3, True, seed=1)
        torch.cuda.synchronize()
        buf = (ctypes.c_ulonglong * 64)()
        lib.dpt_debug_stamps(ctypes.addressof(buf), 64, 0)
        v = np.array(buf[:8], dtype=np.float64)
        tot = v.sum()
        res[f"tile{tile}_H{H}"] = {n: {"cycles_per_step": v[i] / H, "share": v[i] / tot} for i, n in enumerate(names)}
        res[f"tile{tile}_H{H}"]["total_cycles_per_step"] = tot / H
print(json.dumps(res))
