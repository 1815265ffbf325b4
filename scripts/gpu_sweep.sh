#!/bin/bash
# horizon sweep (fixed per-step cost, marginal rate per band) + Infinity-Cache budget sweep
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SW_TILES=8 SW_H=${SW_H:-16,32,64,128,256,384,500} timeout -k 10 300 python scripts/h_sweep.py > gpurun_out/h_sweep.log 2>&1 || exit $?
B=libdpt_hip.so
timeout -k 10 600 python scripts/ab_lib.py ${SWEEP_LIBS:-$B:0 $B:167772160 $B:201326592 $B:234881024 $B:251658240 $B:268435456 $B:301989888} > gpurun_out/ab_budget.log 2>&1
