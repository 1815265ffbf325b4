#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/t_kern.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_kern.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python scripts/ab_tile.py > gpurun_out/ab_tile.log 2>&1 || exit $?
AB_H=1000 AB_A=20 AB_ROUNDS=3 timeout -k 10 600 python scripts/ab_tile.py > gpurun_out/ab_tile_linear.log 2>&1
