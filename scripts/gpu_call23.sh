#!/bin/bash
# DPT_DR_PREFETCH (the next forward's workspace rows issued before the barrier the waves wait at
# during the serial tail and the memo-hit chain) against the product build, config 3
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_WL=darkroom AB_DR_R=1 AB_ROUNDS=5 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_pf.so \
    > gpurun_out/ab23_R1.json 2> gpurun_out/ab23_R1.err
