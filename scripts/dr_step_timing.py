"""DarkRoom online eval at window 201 (H = 200, horizon 100, R = 2; 4096 tasks x 4 episodes): the
fused kernel (8 waves per task for windows up to 256, 16 up to 512) against the per-step device
loop (one window forward per step through dpt_forward_window), each with and without the logits
memo.  Env DR_H, DR_HORIZON, DR_EPS, DR_N change the shape (DR_H=300: window 301, the 16-wave
kernel).  Prints one JSON line."""
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

H, horizon, Heps, N = (int(os.environ.get(k, d)) for k, d in
                        (("DR_H", "200"), ("DR_HORIZON", "100"), ("DR_EPS", "4"), ("DR_N", "4096")))
sd, tm = bench.synthetic_state_dict(4, 2, 5, H)
tm.load_state_dict({**sd, "transformer.wte.weight": tm.transformer.wte.weight}, strict=True)
tm.cuda().eval()
rs = np.random.RandomState(0)
envs = [DarkroomEnv(10, rs.randint(0, 10, 2), horizon) for _ in range(N)]
res = {}
for fused in (True, False):
    for memo in (True, False):
        dpt_hip.set_darkroom_memo(memo)
        times = []
        for _ in range(2):
            np.random.seed(1)
            ctrl = DarkroomTransformerController(tm, batch_size=N, sample=True)
            vec = DarkroomEnvVec(envs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ret = eval_darkroom.deploy_online_vec(vec, ctrl, Heps, H, horizon, fused=fused)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        res[f"{'fused' if fused else 'per_step'}_memo{int(memo)}_s"] = min(times)
        res[f"{'fused' if fused else 'per_step'}_memo{int(memo)}_return_sum"] = int(ret.sum())
dpt_hip.set_darkroom_memo(True)
res["window"] = 1 + H
res["env_steps"] = N * Heps * horizon
print(json.dumps(res))
