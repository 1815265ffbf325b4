"""Classical baseline rollouts (dpt_rollout_policy: evals/eval_bandit.py's Emp / UCB / Thompson /
LCB / LinUCB controllers, ctrls/ctrl_bandit.py) at the bench shapes: 5-arm bandit H = 500 and the
20-arm linear bandit H = 1000 (d = 2), 4096 tasks.  HIP events around each launch, best of 3.
Prints one JSON line of ms per launch and env-steps/s (the wave-per-task kernel; the round-4
lane-per-task kernel was retired in round 6, its timings are in profiles/r5a/policy_timing.jsonl)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import dpt_hip  # noqa: E402

N = 4096
res = {}
rs = np.random.RandomState(0)
cases = [("bandit5_H500", 5, 500, None, rs.uniform(0, 1, (N, 5)))]
arms = rs.normal(size=(20, 2)) / np.sqrt(2)
theta = rs.normal(0, 1, (N, 2)) / np.sqrt(2)
cases.append(("linear20_H1000", 20, 1000, arms, theta @ arms.T))
pols = {"emp": dpt_hip.POLICY_EMP, "ucb": dpt_hip.POLICY_UCB, "thompson": dpt_hip.POLICY_THOMPSON,
        "lcb": dpt_hip.POLICY_LCB, "linucb": dpt_hip.POLICY_LINUCB}
for kern in ("wave",):
    for name, A, H, arm_feats, means in cases:
        for pn, pol in pols.items():
            if pn == "linucb" and arm_feats is None:
                continue
            kw = dict(arms=arm_feats) if pn == "linucb" else {}
            best = None
            for rep in range(4):
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                dpt_hip.rollout_policy(pol, means, H, 0.3, seed=rep, **kw)
                e.record()
                torch.cuda.synchronize()
                if rep:
                    best = min(best or 1e30, a.elapsed_time(e))
            res[f"{kern}/{name}/{pn}"] = {"ms": best, "env_steps_per_s": N * H / (best * 1e-3)}
            print(json.dumps({f"{kern}/{name}/{pn}": res[f"{kern}/{name}/{pn}"]}), flush=True)
print(json.dumps(res))
