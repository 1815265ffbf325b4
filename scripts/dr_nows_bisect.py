"""Diagnostic (GPU): the workspace-free DarkRoom kernel of several library builds against the float64
C oracle on the same injected draws.  Each argument is a package root: a worktree made by
scripts/dr_nows_bisect.sh (scratch/nows/<commit>) or "." for this tree, optionally with
":<library file name>" to load another build of that tree (e.g. .:libdpt_hip_nows0.so).  Every build
runs in its own process, which imports that tree's dpt_hip and bench.  Cases: dim 12 (144 cells: no
per-state table, so the workspace-free kernel runs by default) at windows 101 and 201, and dim 11 with
the workspace switched off, memo on.  Prints one JSON line per build: per case, the largest scaled
logit error against the oracle up to each task's first near-tie draw, and the tasks whose actions
differ before it."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [  # (dim, R, Heps, workspace switch)
    (12, 1, 3, True), (12, 2, 4, True), (11, 1, 3, False), (11, 2, 4, False)]
N, HORIZON = 64, 100


def child(tree, lib, out):
    sys.path[:0] = [os.path.join(tree, "decision-pretrained-transformer_amd"), tree]
    from dpt_hip import _lib
    if lib:
        _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__), lib)
    import bench
    import dpt_hip
    res = {}
    for dim, R, Heps, ws in CASES:
        sd, _ = bench.synthetic_state_dict(4, 2, 5, R * HORIZON)
        m = dpt_hip.DeviceModel(sd, 4, 2, 5, 4 * (1 + R * HORIZON))
        goals = np.random.RandomState(3).randint(0, dim, (N, 2))
        u = np.random.RandomState(4).uniform(size=(Heps * HORIZON, N))
        dpt_hip.set_darkroom_workspace(ws)
        o = m.rollout_darkroom(goals, Heps, HORIZON, R, dim=dim, uniforms=u, want_actions=True, want_logits=True)
        dpt_hip.set_darkroom_workspace(True)
        key = f"dim{dim}_R{R}"
        res[key + "_logits"] = o["logits"].cpu().numpy()
        res[key + "_actions"] = o["actions"].cpu().numpy()
        res[key + "_blob"] = dpt_hip.pack_weights(sd, 4).numpy()
    np.savez(out, **res)


def main():
    sys.path.insert(0, ROOT)
    from oracle import c_oracle
    refs = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for arg in sys.argv[1:]:
        tree, _, lib = arg.partition(":")
        tree = os.path.abspath(tree)
        out = os.path.join(ROOT, "gpurun_out", "nows_" + os.path.basename(tree) + (lib or "") + ".npz")
        cp = subprocess.run([sys.executable, __file__, "--child", tree, lib, out], capture_output=True, text=True,
                            timeout=600)
        if cp.returncode != 0:
            print(json.dumps({"build": arg, "error": cp.stderr[-2000:]}), flush=True)
            sys.exit(cp.returncode)
        d = np.load(out)
        res = {"build": arg}
        for dim, R, Heps, ws in CASES:
            key = f"dim{dim}_R{R}"
            blob = d[key + "_blob"]
            rk = (key, blob.tobytes())
            if rk not in refs:
                u = np.random.RandomState(4).uniform(size=(Heps * HORIZON, N))
                goals = np.random.RandomState(3).randint(0, dim, (N, 2))
                refs[rk] = c_oracle.darkroom_rollout(blob, 4, 4 * (1 + R * HORIZON), goals, Heps, HORIZON, R, u, True,
                                                     dim=dim, threads=16, want_logits=True)
            ref = refs[rk]
            lg, acts = d[key + "_logits"], d[key + "_actions"]
            err, bad_tasks = 0.0, 0
            per_ep = np.zeros(Heps)
            for j in range(N):
                tie = np.nonzero(ref["margin"][:, j] < 1e-5)[0]
                n = int(tie[0]) if tie.size else Heps * HORIZON
                k = min(n + 1, Heps * HORIZON)
                e = np.abs(lg[:k, j] - ref["logits"][:k, j]) / np.maximum(1.0, np.abs(ref["logits"][:k, j]))
                err = max(err, float(e.max()))
                per_ep_j = [float(e[ep * HORIZON:min(k, (ep + 1) * HORIZON)].max(initial=0.0)) for ep in range(Heps)]
                per_ep = np.maximum(per_ep, per_ep_j)
                bad_tasks += int(not np.array_equal(acts[j, :n], ref["actions"][j, :n]))
            res[key] = {"max_scaled_logit_err": err, "per_episode": [float(x) for x in per_ep],
                        "tasks_with_action_mismatch": bad_tasks}
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        main()
