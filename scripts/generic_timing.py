"""Timing of the generic-width bandit rollout (dpt_rollout_bandit_generic) at the C2 shape
(4096 tasks x H = 500, 5 arms, L = 4) for several widths, beside the fused E = 32 kernel and the
per-step path it replaces (Transformer.forward over the whole window every step, timed on a
short horizon).  Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
from dpt_hip import train as tr  # noqa: E402
from models.net import Transformer  # noqa: E402


def model(E, L, H):
    torch.manual_seed(E)
    m = Transformer(dict(horizon=H, state_dim=1, action_dim=5, n_layer=L, n_embd=E, n_head=1, dropout=0.0,
                         test=True)).cuda().eval()
    return m


def timed(fn, reps=2):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    N, H, L = int(os.environ.get("GT_N", 4096)), int(os.environ.get("GT_H", 500)), 4
    means = np.random.RandomState(0).uniform(0, 1, (N, 5))
    out = {"N": N, "H": H, "L": L}
    widths = [int(w) for w in os.environ.get("GT_E", "16,32,48,64,128").split(",")]
    for E in widths:
        m = model(E, L, H)
        t = timed(lambda: tr.rollout_bandit_generic(m, means, H, 0.3, True, seed=1))
        out[f"generic_E{E}"] = {"s": t, "env_steps_per_s": N * H / t}
        if E == 32:
            dm = m.device_model()
            t = timed(lambda: dm.rollout_bandit(means, H, 0.3, True, seed=1))
            out["fused_E32"] = {"s": t, "env_steps_per_s": N * H / t}
        print(json.dumps({k: v for k, v in out.items() if k.endswith(f"E{E}")}), file=sys.stderr, flush=True)
    if os.environ.get("GT_PER_STEP", "1") != "1":
        print(json.dumps(out))
        return
    # the per-step path at width 64 (what the generic rollout replaces), short horizon
    from ctrls.ctrl_bandit import BanditTransformerController
    from envs.bandit_env import BanditEnv, BanditEnvVec
    from evals import eval_bandit
    Hs, Ns = 50, 1024
    m = model(64, L, H)
    vec = BanditEnvVec([BanditEnv(mu, Hs, var=0.3) for mu in means[:Ns]])
    ctrl = BanditTransformerController(m, sample=True, batch_size=Ns)
    t = timed(lambda: eval_bandit.deploy_online_vec(vec, ctrl, Hs, fused=False), reps=1)
    out["per_step_E64_H50_N1024"] = {"s": t, "env_steps_per_s": Ns * Hs / t}
    m2 = model(64, L, H)
    t = timed(lambda: tr.rollout_bandit_generic(m2, means[:Ns], Hs, 0.3, True, seed=1))
    out["generic_E64_H50_N1024"] = {"s": t, "env_steps_per_s": Ns * Hs / t}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
