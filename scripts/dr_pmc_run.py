"""One config-3-width DarkRoom rollout (4096 tasks, window 101, memo off unless DR_MEMO=1, DR_EPS episodes, default 10) on the
library named by argv[1] (a file in dpt_hip/), for per-variant PMC passes (scripts/dr_pmc_variants.sh):
prints the number of window forwards the launch ran, the divisor of the per-forward counters."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
from dpt_hip import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__), sys.argv[1])
import bench  # noqa: E402
import dpt_hip  # noqa: E402

sd, _ = bench.synthetic_state_dict(4, 2, 5, 100)
m = dpt_hip.DeviceModel(sd, 4, 2, 5, 404)
dpt_hip.set_darkroom_memo(os.environ.get("DR_MEMO", "0") == "1")  # memo off: every step one forward
goals = np.array([(j, i) for j in range(10) for i in range(10)])
np.random.RandomState(0).shuffle(goals)
goals = goals[np.arange(4096) % 100]
o = m.rollout_darkroom(goals, int(os.environ.get("DR_EPS", "10")), 100, 1, seed=1, want_forwards=True)
torch.cuda.synchronize()
print("forwards", int(o["forwards"].to(torch.int64).sum()))
