#!/bin/bash
# DarkRoom config 3: four workgroups per CU (LDS now fits: embedding from global memory) with and
# without sequential blocks, against the default three
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_WL=darkroom AB_DR_R=1 AB_ROUNDS=3 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_embg.so \
    libdpt_hip_wg4.so libdpt_hip_wg4seq.so > gpurun_out/ab6.json 2> gpurun_out/ab6.err
