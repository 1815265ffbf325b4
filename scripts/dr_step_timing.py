"""Per-step DarkRoom device loop (window 201 > 128: not fused) with and without the logits memo."""
import os, sys, time, numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import bench, dpt_hip
from ctrls.ctrl_darkroom import DarkroomTransformerController
from envs.darkroom_env import DarkroomEnv, DarkroomEnvVec
from evals import eval_darkroom
sd, tm = bench.synthetic_state_dict(4, 2, 5, 200)
tm.load_state_dict({**sd, "transformer.wte.weight": tm.transformer.wte.weight}, strict=True); tm.cuda()
rs = np.random.RandomState(0)
envs = [DarkroomEnv(10, rs.randint(0, 10, 2), 100) for _ in range(4096)]
for memo in (False, True, False, True):
    dpt_hip.set_darkroom_memo(memo)
    np.random.seed(1)
    ctrl = DarkroomTransformerController(tm, batch_size=4096, sample=True)
    vec = DarkroomEnvVec(envs)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    ret = eval_darkroom.deploy_online_vec(vec, ctrl, 4, 200, 100)
    torch.cuda.synchronize(); dt = time.perf_counter() - t0
    print("memo", memo, "per-step path, R=2, 4096 tasks x 4 eps x 100 steps:", round(dt, 3), "s", ret.sum())
