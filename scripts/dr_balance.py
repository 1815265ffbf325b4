"""Per-task work of the config-3 DarkRoom rollout (window forwards per task, summed over the
episodes): the spread sets how much of the last wave of workgroups idles at the end."""
import json
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
N = 4096
goals = np.array([(j, i) for j in range(10) for i in range(10)])
np.random.RandomState(0).shuffle(goals)
goals = goals[np.arange(N) % 100]
out = m.rollout_darkroom(goals, 40, 100, 1, seed=3, want_forwards=True)
torch.cuda.synchronize()
fw = out["forwards"].cpu().numpy().sum(1).astype(np.float64)
q = np.percentile(fw, [0, 10, 50, 90, 99, 100])
by_goal = [float(fw[np.arange(N) % 100 == g].mean()) for g in range(100)]
print(json.dumps({"mean": fw.mean(), "std": fw.std(), "pct_0_10_50_90_99_100": q.tolist(),
                  "goal_mean_min_max": [min(by_goal), max(by_goal)],
                  "goal_explained_var": float(np.var(np.array(by_goal)[np.arange(N) % 100]) / fw.var())}))
