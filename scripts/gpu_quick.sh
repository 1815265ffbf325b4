#!/bin/bash
# quick iteration: every GPU test, then the headline bench line (no CPU baseline)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/bench_quick.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload linear --steps 2 --warmup 1 > gpurun_out/bench_quick_linear.log 2>&1
