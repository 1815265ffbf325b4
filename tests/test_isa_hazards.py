"""Every kernel's machine code keeps the MFMA (and VALU) wait states on every control-flow path.

hipcc's hazard recognizer (ROCm 7.2, gfx950) sets the wait states between a v_mfma and the VALU /
LDS instructions that read or overwrite its registers; across basic blocks it can count too few
(a consumer reached through a taken branch 2-7 issue slots after the MFMA, where straight-line code
keeps 8).  Such a read returns the register's old contents or not, depending on timing: the
symptom is a nondeterministic wrong result (a first-pair peel in attend gave NaN logits through one
such path).  scripts/isa_hazard_cfg.py walks every path of every kernel and compares the distances
with the smallest ones the compiler keeps in straight-line code; the sources are written so that no
path comes closer (attend's branch-free masked tiles, the layer-0 query projection after the token-0
store).  The scan also applies the VALU rules (2 wait states before an MFMA or v_permlane reads a
VALU result, 1 before v_readlane, 1 after a transcendental).  CPU only: hipcc -S for gfx950."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "decision-pretrained-transformer_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def file_flags(src):
    """the Makefile's per-file code-generation flags (FLAGS_<name> := ...) for this source"""
    name = src.rsplit(".", 1)[0]
    for line in open(os.path.join(CSRC, "Makefile")):
        if line.startswith(f"FLAGS_{name} :="):
            return line.split(":=", 1)[1].split()
    return []


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", ["dpt_darkroom.hip", "dpt_prefill.hip", "dpt_decode.hip", "dpt_train.hip",
                                 "dpt_policies.hip", "dpt_env.hip", "dpt_stats.hip", "dpt_abi.hip"])
def test_no_short_mfma_hazard_paths(src, tmp_path):
    import isa_hazard_cfg
    out = tmp_path / (src + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-slp-vectorize",
                    "-I" + os.path.join(ROOT, "include"), *file_flags(src), "--cuda-device-only", "-S",
                    os.path.join(CSRC, src), "-o", str(out)], check=True, capture_output=True)
    isa_hazard_cfg.ALL_PRODUCERS = True  # the VALU rules too (-> MFMA / permlane / readlane, transcendental)
    assert isa_hazard_cfg.scan_all([str(out)]) == 0


def test_scanner_finds_a_short_path(tmp_path):
    """the scanner itself: an MFMA result read 2 slots later through a taken branch is reported"""
    import isa_hazard_cfg
    s = tmp_path / "k.s"
    s.write_text("""_Z1kv:
\tv_mfma_f32_16x16x32_f16 v[6:9], v[2:5], v[10:13], 0
\ts_nop 7
\tv_add_f32_e32 v20, v6, v7
\tv_mfma_f32_16x16x32_f16 v[6:9], v[2:5], v[10:13], 0
\ts_cbranch_vccnz .LBB0_2
\ts_nop 7
\tv_mov_b32_e32 v8, 0
.LBB0_2:
\tv_add_f32_e32 v21, v8, v9
\ts_endpgm
.Lfunc_end0:
""")
    isa_hazard_cfg.ALL_PRODUCERS = False
    assert isa_hazard_cfg.scan_all([str(s)]) == 1
    # a VALU write read by a cross-lane permute 1 slot later on the branch path, a transcendental's
    # result read at once
    v = tmp_path / "v.s"
    v.write_text("""_Z1vv:
\tv_add_f32_e32 v2, v3, v4
\ts_cbranch_vccnz .LBB0_2
\ts_nop 1
.LBB0_2:
\tv_permlane32_swap_b32_e32 v2, v5
\tv_exp_f32_e32 v7, v8
\tv_add_f32_e32 v9, v7, v7
\ts_endpgm
.Lfunc_end0:
""")
    isa_hazard_cfg.ALL_PRODUCERS = True
    assert isa_hazard_cfg.scan_all([str(v)]) == 2
