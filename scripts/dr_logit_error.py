"""Largest logit error of the fused DarkRoom rollout against the reference's recorded
logits (tests/golden rollout_darkroom_*.npz), in units of max(1, |x|): the margin left
under the 1e-5 parity bar.  Test infrastructure (reads the golden fixtures)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "decision-pretrained-transformer_amd")]
from dpt_hip import _lib  # noqa: E402

if os.environ.get("DPT_LIB"):  # another build in dpt_hip/ (A/B)
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__), os.environ["DPT_LIB"])
from conftest import golden  # noqa: E402
from oracle import dpt_oracle as O  # noqa: E402
from test_gpu_kernels import model_from_golden  # noqa: E402

out = {}
_, m, _ = model_from_golden("darkroom")
for tag in ("sample", "greedy", "permuted"):
    r = golden(f"rollout_darkroom_{tag}.npz")
    n, Heps, H, horizon, sample = (int(x) for x in r["cfg"])
    perms = O.perm_table()[r["perm_index"]] if tag == "permuted" else None
    o = m.rollout_darkroom(r["goals"], Heps, horizon, H // horizon, perms=perms, sample=bool(sample),
                           uniforms=r["u"].reshape(-1, n), want_actions=True, want_logits=True)
    lg, ref = o["logits"].cpu().numpy(), r["logits"]
    err = np.abs(lg - ref) / np.maximum(1.0, np.abs(ref))
    out[tag] = {"max_scaled_err": float(err.max()), "mean_scaled_err": float(err.mean()),
                "returns_equal": bool(np.array_equal(o["returns"].cpu().numpy(), r["returns"]))}
print(json.dumps(out))
