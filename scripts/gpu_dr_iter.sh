#!/bin/bash
# darkroom iteration: parity tests -> phase stamps -> bench line
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -x -q -m gpu -k "darkroom" > gpurun_out/t_dr.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_dr.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python scripts/dr_stamps.py > gpurun_out/dr_stamps.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload darkroom --steps 2 --warmup 1 > gpurun_out/bench_dr.log 2>&1
