"""Logit error of the MFMA prefill (fp16 two-part split products) and of the fp32
position-by-position path against the float64 oracle, on the DarkRoom fixture model with its
block weights scaled by a factor (LayerNorm gains x3 for factors > 1): how the split
products' accuracy compares with fp32's as the scores and activations grow."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
import dpt_hip  # noqa: E402
from oracle import dpt_oracle as O  # noqa: E402

g = dict(np.load(os.path.join(ROOT, "tests", "golden", "forward_darkroom.npz")))
H, sd, A, L, E = (int(x) for x in g["cfg"])
res = {}
for factor in [float(f) for f in os.environ.get("FACTORS", "0.015625 1 2 4 8").split()]:
    w = {}
    for k, v in g.items():
        if not k.startswith("w/"):
            continue
        t = v.astype(np.float32).copy()
        if any(s in k for s in ("c_fc.weight", "c_proj.weight", "c_attn.weight")):
            t *= factor
        if factor > 1 and ("ln_1.weight" in k or "ln_2.weight" in k):
            t *= 3.0
        w[k[2:]] = t
    m = dpt_hip.DeviceModel({k: torch.from_numpy(v) for k, v in w.items()}, L, sd, A, 4 * (1 + H))
    W = O.split_weights(w, L)
    rs = np.random.RandomState(31)
    N, C = 32, 100
    q = rs.randn(N, sd).astype(np.float32)
    cs, cn = rs.randn(N, C, sd).astype(np.float32), rs.randn(N, C, sd).astype(np.float32)
    ca = np.eye(A, dtype=np.float32)[rs.randint(0, A, (N, C))]
    cr = rs.randn(N, C).astype(np.float32)
    ref = O.transformer_forward(W, q, cs, ca, cn, cr, test=True)
    out = {}
    for on in (True, False):
        dpt_hip.set_prefill(on)
        lg = m.forward_window(q, cs, ca, cn, cr, out_mode=0).cpu().numpy().astype(np.float64)
        out["prefill_fp16x3" if on else "positionwise_fp32"] = float(
            (np.abs(lg - ref) / np.maximum(1.0, np.abs(ref))).max())
    dpt_hip.set_prefill(True)
    out["max_abs_logit"] = float(np.abs(ref).max())
    res[factor] = out
    print(factor, out, flush=True)
print(json.dumps(res))
