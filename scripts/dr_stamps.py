"""Per-phase cycles of one DarkRoom step (diagnostic build libdpt_hip_stamps.so), config 3 width."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
from dpt_hip import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__),
                             os.environ.get("DPT_STAMPS_LIB", "libdpt_hip_stamps.so"))
lib = _lib.load()
lib.dpt_debug_dr_stamps.restype = ctypes.c_int
lib.dpt_debug_dr_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

L = 4
sd, _ = bench.synthetic_state_dict(L, 2, 5, 100)
m = dpt_hip.DeviceModel(sd, L, 2, 5, 404)
dpt_hip.set_darkroom_memo(bool(int(os.environ.get("DR_MEMO", "0"))))  # per-forward costs: memo off
Heps = 11  # episode 0 (window 1) is 1/11 of the steps
names = ["L0:embed+query k/v", "L0:merge+c_proj+mlp (wave 0 view)"]
for layer in range(1, L - 1):
    names += [f"L{layer}:ln1+c_attn (+prev mlp)", f"L{layer}:attn+c_proj"]
names += [f"L{L - 1}:ln1+c_attn (+prev mlp)", "tail1:key-tile partials", "tail2:merge+c_proj+mlp chunk",
          "tail3:barrier after select", "tail3a:part_y+ln_f+head", "tail3b:cdf+select+env (lane 0)",
          "memo hits + barrier"]
out = {}
for N in (256, 512, 4096):
    goals = np.stack(np.unravel_index(np.arange(N) % 100, (10, 10)), 1)
    m.rollout_darkroom(goals, Heps, 100, 1, seed=0)
    torch.cuda.synchronize()
    lib.dpt_debug_dr_stamps(None, 0, 1)
    t0 = time.perf_counter()
    m.rollout_darkroom(goals, Heps, 100, 1, seed=1)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    buf = (ctypes.c_ulonglong * 32)()
    lib.dpt_debug_dr_stamps(ctypes.addressof(buf), 32, 0)
    v = np.array(buf[:2 * L + 5], dtype=np.float64) / (Heps * 100)
    res = {n: round(float(x)) for n, x in zip(names, v) if x > 0}
    res["total_cycles_per_step"] = round(float(v.sum()))
    res["wall_s"] = dt
    res["env_steps_per_s"] = N * Heps * 100 / dt
    out[N] = res
print(json.dumps(out))
