#!/bin/bash
# the r6b evidence pass on the final code, then per-phase instruction counts of the DarkRoom kernel
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_evidence.sh r6b || exit $?
bash scripts/dr_pmc_variants.sh libdpt_hip.so libdpt_hip_skipmlp.so libdpt_hip_skipattn.so libdpt_hip_skiptail.so \
    libdpt_hip_skipall.so
