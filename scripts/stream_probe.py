"""Runs scripts/stream_probe.hip (a code object built here with hipcc --genco into scripts/stream_probe.co if absent):
the bandit rollout's y-stream read pattern at config 2 (4096 tasks, H=500, 3 streamed blocks),
no compute.  Prints the time and the algorithmic y bytes / time for a few residency budgets."""
import ctypes
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "stream_probe.co")
if not os.path.exists(SO):
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--genco", "--offload-arch=gfx950", "-O3",
                           os.path.join(HERE, "stream_probe.hip"), "-o", SO])
N, H, nblk = int(os.environ.get("SP_N", "4096")), int(os.environ.get("SP_H", "500")), 3
y = torch.zeros(nblk * N * H * 32, dtype=torch.float32, device="cuda")
out = torch.zeros(1, device="cuda")
mod = ctypes.c_void_p()
hip = ctypes.CDLL("libamdhip64.so")
assert hip.hipModuleLoad(ctypes.byref(mod), SO.encode()) == 0
res = {}
row = N * 32 * 4  # one position of one block, all tasks
for kname in ("stream_probe", "stream_probe_r16", "stream_probe_r4", "stream_probe_nosync", "stream_probe_temporal"):
    fn = ctypes.c_void_p()
    assert hip.hipModuleGetFunction(ctypes.byref(fn), mod, kname.encode()) == 0
    for mib in ((0, 224) if kname == "stream_probe" else (224,)):
        pin = min(H, (mib << 20) // (row * nblk))
        args = [ctypes.c_void_p(y.data_ptr()), ctypes.c_int(N), ctypes.c_int(H), ctypes.c_int(pin), ctypes.c_int(nblk),
                ctypes.c_void_p(out.data_ptr())]
        ptrs = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.pointer(a), ctypes.c_void_p) for a in args])
        ts = []
        for rep in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert hip.hipModuleLaunchKernel(fn, N // 8, 1, 1, 512, 1, 1, 0, None, ptrs, None) == 0
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = min(ts)
        by = nblk * 128 * N * H * (H - 1) / 2
        res[f"{kname}@{mib}MiB"] = {"pin": pin, "ms": ms, "TBps": by / ms / 1e9}
        print(json.dumps({kname: res[f"{kname}@{mib}MiB"]}), flush=True)
print(json.dumps(res))
