"""Register / scratch budget of the two bench kernels, from hipcc's kernel-resource-usage remarks
(gfx950, the Makefile's flags including its per-file ones).  CPU only.

- rollout_darkroom_kernel<true, 4, true> (config 3): no scratch and at most 168 VGPRs, so three
  4-wave workgroups share a CU (DarkRoom);
- rollout_bandit_kernel<8, *, 0> (config 2, the default vector form of block 0): no scratch and
  four waves per SIMD."""
import os
import re
import subprocess

import pytest

from test_isa_hazards import CSRC, HIPCC, ROOT, file_flags


def remarks(src, tmp_path):
    cp = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=off",
                         "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"), *file_flags(src),
                         "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, src),
                         "-o", str(tmp_path / "k.o")], capture_output=True, text=True, check=True)
    out, cur = {}, None
    for line in cp.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        for key, short in (("VGPRs", "vgpr"), ("ScratchSize [bytes/lane]", "scratch"),
                           ("Occupancy [waves/SIMD]", "occ")):
            m = re.search(re.escape(key) + r": (\d+)", line)
            if m and cur is not None:
                cur[short] = int(m.group(1))
    return out


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_darkroom_config3_kernel_budget(tmp_path):
    r = remarks("dpt_darkroom.hip", tmp_path)
    k = [v for n, v in r.items() if "rollout_darkroom_kernelILb1ELi4ELb1E" in n]
    assert len(k) == 1, list(r)
    assert k[0]["scratch"] == 0 and k[0]["vgpr"] <= 168 and k[0]["occ"] >= 3, k[0]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_bandit_config2_kernel_budget(tmp_path):
    r = remarks("dpt_decode.hip", tmp_path)
    k = [v for n, v in r.items() if re.search(r"rollout_bandit_kernelILi8ELb[01]ELi0E", n)]
    assert len(k) == 2, list(r)
    for v in k:
        assert v["scratch"] == 0 and v["occ"] >= 4, v
