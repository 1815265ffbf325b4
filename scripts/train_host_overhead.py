"""Host-side cost of one training step (train.py:286-331 shape, DarkRoom T = 101 and bandit T = 501,
batch 64): the time to enqueue the step without waiting for the device, split into the two
library calls (dpt_train_forward / dpt_train_backward launch sequences) and the rest (Python,
autograd, parameter packing, loss, AdamW).  Prints one JSON line."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT, os.path.join(ROOT, "scripts")]
from models.net import Transformer  # noqa: E402
import dpt_hip.train as tr  # noqa: E402
from train_timing import batch  # noqa: E402

acc = {"forward": 0.0, "backward": 0.0}
_f, _b = tr.forward, tr.backward


def fwd(*a):
    t = time.perf_counter()
    r = _f(*a)
    acc["forward"] += time.perf_counter() - t
    return r


def bwd(*a):
    t = time.perf_counter()
    r = _b(*a)
    acc["backward"] += time.perf_counter() - t
    return r


tr.forward, tr.backward = fwd, bwd
res = {}
dev = torch.device("cuda")
for name, sd, A, H in (("bandit_T501", 1, 5, 500), ("darkroom_T101", 2, 5, 100)):
    torch.manual_seed(0)
    m = Transformer(dict(horizon=H, state_dim=sd, action_dim=A, n_layer=4, n_embd=32, n_head=1, dropout=0.0,
                         test=False)).to(dev).train()
    b = batch(64, H, sd, A, dev, np.random.RandomState(0))
    ce = torch.nn.CrossEntropyLoss(reduction="sum")
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    true = b["optimal_actions"][:, None, :].expand(64, H, A).reshape(-1, A)

    def step():
        pred = m(b)
        loss = ce(pred.reshape(-1, A), true)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    reps = 20
    acc["forward"] = acc["backward"] = 0.0
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        step()
        host += time.perf_counter() - t
        torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / reps
    res[name] = {"host_enqueue_ms": host / reps * 1e3, "lib_forward_ms": acc["forward"] / reps * 1e3,
                 "lib_backward_ms": acc["backward"] / reps * 1e3, "synced_step_ms": wall * 1e3}
print(json.dumps(res))
