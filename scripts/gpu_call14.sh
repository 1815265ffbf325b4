#!/bin/bash
# historic build 3c9b0eb (workspace-free step specialised; logits 5.3e-2 off at window 201 in the
# r6 bisect) against the same build with only the layer-0 query projection moved after the token-0
# store (no MFMA read through a branch: scripts/isa_hazard_cfg.py), both against the float64 oracle
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python scripts/dr_nows_bisect.py scratch_run/3c9b0eb_src scratch_run/3c9b0eb_src:libdpt_hip_fix.so \
    > gpurun_out/nows_fix.jsonl 2> gpurun_out/nows_fix.err
