#!/bin/bash
# A/B of library builds at config 2 and at the linear config's per-GPU width (A=20, H=1000)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/ab_lib.py $AB_LIBS > gpurun_out/ab_c2.log 2>&1 || exit $?
if [ -n "$AB_LINEAR" ]; then
  AB_A=20 AB_H=1000 timeout -k 10 600 python scripts/ab_lib.py $AB_LIBS > gpurun_out/ab_lin.log 2>&1 || exit $?
fi
if [ -n "$AB_SWEEP" ]; then
  SW_TILES=8 SW_H=16,32,64,128,256,384,500 timeout -k 10 300 python scripts/h_sweep.py > gpurun_out/h_sweep.log 2>&1
fi
