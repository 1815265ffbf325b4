"""A short DarkRoom rollout at the config-3 width (4096 tasks, window 101, memo on) for PC sampling
(scripts/pc_sample_darkroom.sh): one warm launch, then DR_EPS episodes (default 6) under the sampler."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

L = 4
sd, _ = bench.synthetic_state_dict(L, 2, 5, 100)
m = dpt_hip.DeviceModel(sd, L, 2, 5, 404)
goals = np.array([(j, i) for j in range(10) for i in range(10)])
np.random.RandomState(0).shuffle(goals)
goals = goals[np.arange(4096) % 100]
eps = int(os.environ.get("DR_EPS", "6"))
m.rollout_darkroom(goals, 2, 100, 1, seed=0)
torch.cuda.synchronize()
o = m.rollout_darkroom(goals, eps, 100, 1, seed=1)
torch.cuda.synchronize()
print("returns", int(o["returns"].sum()))
