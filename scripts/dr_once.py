"""One DarkRoom online evaluation at config-3 width (profiling target): 4096 tasks, 11 episodes."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402

sd, _ = bench.synthetic_state_dict(4, 2, 5, 100)
m = dpt_hip.DeviceModel(sd, 4, 2, 5, 404)
goals = np.stack(np.unravel_index(np.arange(4096) % 100, (10, 10)), 1)
m.rollout_darkroom(goals, 11, 100, 1, seed=1)
torch.cuda.synchronize()
print("ok")
