"""Diagnostic: the workspace-free DarkRoom kernel (set_darkroom_workspace(False)) against the
workspace kernel on the same draws, per library build (argv), memo off: largest logit difference per
episode.  Used to chase the workspace-free step specialisation (DPT_DR_SPEC_NOWS)."""
import json
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

dim = int(os.environ.get("DR_DIM", "10"))
R, horizon, Heps, N = int(os.environ.get("DR_R", "1")), 100, 3, 64
sd, _ = bench.synthetic_state_dict(4, 2, 5, R * horizon)
m = dpt_hip.DeviceModel(sd, 4, 2, 5, 4 * (1 + R * horizon))
goals = np.random.RandomState(3).randint(0, dim, (N, 2))
dpt_hip.set_darkroom_memo(False)
u = np.random.RandomState(4).uniform(size=(Heps * horizon, N))
outs = {}
for ws in (True, False):
    dpt_hip.set_darkroom_workspace(ws)
    o = m.rollout_darkroom(goals, Heps, horizon, R, dim=dim, uniforms=u, want_actions=True, want_logits=True)
    outs[ws] = {k: o[k].cpu().numpy() for k in ("actions", "logits")}
dpt_hip.set_darkroom_workspace(True)
a, b = outs[True], outs[False]
res = {"lib": sys.argv[1], "dim": dim}
# the float64 C oracle on a few tasks, same draws (the workspace-free run): largest logit error per episode
sys.path.insert(0, ROOT)
from oracle import c_oracle  # noqa: E402
tasks = np.arange(0, N, 8)
ref = c_oracle.darkroom_rollout(dpt_hip.pack_weights(sd, 4).numpy(), 4, 4 * (1 + R * horizon), goals[tasks], Heps,
                                horizon, R, u[:, tasks], True, dim=dim, threads=16, want_logits=True)
rl = np.asarray(ref["logits"])  # (steps, tasks, A)
ra = np.asarray(ref["actions"])
for ep in range(Heps):
    sl = slice(ep * horizon, (ep + 1) * horizon)
    same = (b["actions"][tasks][:, sl] == ra[:, sl]).all(1)
    d = np.abs(b["logits"][sl][:, tasks] - rl[sl]) / np.maximum(1.0, np.abs(rl[sl]))
    res[f"oracle_ep{ep}"] = {"max_scaled_err_same_tasks": float(d[:, same].max()) if same.any() else None,
                             "tasks_same_actions": int(same.sum())}
for ep in range(Heps):
    sl = slice(ep * horizon, (ep + 1) * horizon)
    same = (a["actions"][:, sl] == b["actions"][:, sl]).all(1)
    d = np.abs(a["logits"][sl] - b["logits"][sl])  # (steps, N, A)
    res[f"ep{ep}"] = {"max_logit_diff_same_tasks": float(d[:, same].max()) if same.any() else None,
                      "tasks_same_actions": int(same.sum())}
print(json.dumps(res))
