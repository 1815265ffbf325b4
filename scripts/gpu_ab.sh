#!/bin/bash
# library A/B (Makefile variants) + phase stamps of the shipped configuration
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/ab_lib.py ${AB_LIBS:-libdpt_hip.so libdpt_hip_y6.so libdpt_hip_y8.so} > gpurun_out/ab_lib.log 2>&1 || exit $?
if [ -n "$AB_STAMPS" ]; then timeout -k 10 300 python scripts/phase_stamps.py > gpurun_out/stamps.log 2>&1; fi
