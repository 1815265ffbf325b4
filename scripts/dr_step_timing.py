"""DarkRoom online eval at window 201 (H = 200, horizon 100, R = 2; 4096 tasks x 4 episodes): the
fused 8-wave kernel (windows up to 256) against the per-step device loop (one window forward per
step through dpt_forward_window), each with and without the logits memo.  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench  # noqa: E402
import dpt_hip  # noqa: E402
from ctrls.ctrl_darkroom import DarkroomTransformerController  # noqa: E402
from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec  # noqa: E402
from evals import eval_darkroom  # noqa: E402

sd, tm = bench.synthetic_state_dict(4, 2, 5, 200)
tm.load_state_dict({**sd, "transformer.wte.weight": tm.transformer.wte.weight}, strict=True)
tm.cuda().eval()
rs = np.random.RandomState(0)
envs = [DarkroomEnv(10, rs.randint(0, 10, 2), 100) for _ in range(4096)]
res = {}
for fused in (True, False):
    for memo in (True, False):
        dpt_hip.set_darkroom_memo(memo)
        times = []
        for _ in range(2):
            np.random.seed(1)
            ctrl = DarkroomTransformerController(tm, batch_size=4096, sample=True)
            vec = DarkroomEnvVec(envs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ret = eval_darkroom.deploy_online_vec(vec, ctrl, 4, 200, 100, fused=fused)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        res[f"{'fused' if fused else 'per_step'}_memo{int(memo)}_s"] = min(times)
        res[f"{'fused' if fused else 'per_step'}_memo{int(memo)}_return_sum"] = int(ret.sum())
dpt_hip.set_darkroom_memo(True)
res["env_steps"] = 4096 * 4 * 100
print(json.dumps(res))
