#!/bin/bash
# quick iteration: kernel parity tests + H sweep + tile A/B + phase stamps
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/t_kern.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python scripts/h_sweep.py > gpurun_out/h_sweep.log 2>&1 || exit $?
timeout -k 10 600 python scripts/ab_tile.py > gpurun_out/ab_tile.log 2>&1 || exit $?
timeout -k 10 600 python scripts/phase_stamps.py > gpurun_out/stamps.log 2>&1
