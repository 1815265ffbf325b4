"""A/B of library builds (Makefile `variants`): one bandit rollout timing per library,
each in its own process (python scripts/ab_lib.py libA.so libB.so ...; rounds alternate).
An argument libX.so:<bytes> runs libX.so with dpt_hip.set_cache_budget(<bytes>); a suffix +b0 / +nob0
runs it with dpt_hip.set_block0_mfma(True / False); +nows / +nomemo run DarkRoom without the
layer-0 workspace / the logits memo (suffixes in that order: lib.so+nows+nomemo).
Env: AB_H, AB_N, AB_A, AB_TILE, AB_ROUNDS."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib):
    sys.path[:0] = [os.path.join(ROOT, "decision-pretrained-transformer_amd"), ROOT]
    from dpt_hip import _lib
    b0 = None  # "libX.so+b0" / "+nob0": DPT_TUNE_BLOCK0_MFMA 1 / 0
    for suf, on in (("+nob0", False), ("+b0", True)):
        if lib.endswith(suf):
            lib, b0 = lib[: -len(suf)], on
    nomemo = lib.endswith("+nomemo")  # DarkRoom with every step a window forward
    lib = lib[: -len("+nomemo")] if nomemo else lib
    nows = lib.endswith("+nows")  # DarkRoom without the per-episode layer-0 workspace
    lib = lib[: -len("+nows")] if nows else lib
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.__file__), lib.split(":")[0])
    import torch
    import bench
    import dpt_hip
    H, N, A = (int(os.environ.get(k, d)) for k, d in (("AB_H", "500"), ("AB_N", "4096"), ("AB_A", "5")))
    dpt_hip.set_decode_tile(int(os.environ.get("AB_TILE", "8")))
    if b0 is not None:
        dpt_hip.set_block0_mfma(b0)
    if nomemo:
        dpt_hip.set_darkroom_memo(False)
    if nows:
        dpt_hip.set_darkroom_workspace(False)
    if ":" in lib:  # "libX.so:<bytes>": the same library at another DPT_TUNE_CACHE_BUDGET
        dpt_hip.set_cache_budget(int(lib.split(":")[1]))
    if os.environ.get("AB_WL") == "darkroom":  # config 3: 4096 tasks x 40 episodes x 100 steps
        # AB_DR_R: context episodes (window 1 + 100 R; 1 = config 3)
        R = int(os.environ.get("AB_DR_R", "1"))
        sd, _ = bench.synthetic_state_dict(4, 2, 5, 100 * R)
        m = dpt_hip.DeviceModel(sd, 4, 2, 5, 4 * (1 + 100 * R))
        goals = np.stack(np.unravel_index(np.arange(N) % 100, (10, 10)), 1)
        ts = []
        for rnd in range(3):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = m.rollout_darkroom(goals, 40, 100, R, seed=rnd)
            b.record()
            torch.cuda.synchronize()
            if rnd > 0:
                ts.append(a.elapsed_time(b))
        # bit-identity digest: actions and logits of a smaller launch (AB_DIGEST=0 skips it)
        digest = None
        if os.environ.get("AB_DIGEST", "1") == "1":
            import hashlib
            o = m.rollout_darkroom(goals[:512], 6, 100, R, seed=77, want_actions=True, want_logits=True)
            h = hashlib.sha1(o["actions"].cpu().numpy().tobytes())
            h.update(o["logits"].cpu().numpy().tobytes())
            digest = h.hexdigest()[:16]
        print(json.dumps({"lib": lib, "ms": ts, "checksum": float(out["returns"].sum()), "digest": digest}))
        return
    sd, _ = bench.synthetic_state_dict(4, 1, A, H)
    m = dpt_hip.DeviceModel(sd, 4, 1, A, 4 * (1 + H))
    means = torch.from_numpy(np.random.RandomState(1).uniform(0, 1, (N, A))).cuda()
    ts = []
    for rnd in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = m.rollout_bandit(means, H, 0.3, True, seed=rnd)
        b.record()
        torch.cuda.synchronize()
        if rnd > 0:
            ts.append(a.elapsed_time(b))
    chk = float(out["arm_value"].sum())
    print(json.dumps({"lib": lib, "ms": ts, "checksum": chk}))


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        sys.exit(0)
    res = {lib: [] for lib in sys.argv[1:]}
    chk = {}
    for rnd in range(int(os.environ.get("AB_ROUNDS", "2"))):
        for lib in sys.argv[1:]:
            cp = subprocess.run([sys.executable, __file__, "--child", lib], capture_output=True, text=True,
                                timeout=300)
            if cp.returncode:
                sys.exit(f"{lib}: child failed ({cp.returncode})\n{cp.stderr[-3000:]}")
            out = cp.stdout.strip().splitlines()[-1]
            d = json.loads(out)
            res[lib] += d["ms"]
            chk[lib] = (d["checksum"], d.get("digest"))
    H, N = int(os.environ.get("AB_H", "500")), int(os.environ.get("AB_N", "4096"))
    sys.path[:0] = [ROOT]
    import bench
    ab = bench.algorithmic_bytes(N, H, 4)
    print(json.dumps({lib: {"median_ms": float(np.median(v)), "min_ms": float(np.min(v)),
                            "TBps": ab / (np.median(v) * 1e-3) / 1e12, "checksum": chk[lib]}
                      for lib, v in res.items()}))
