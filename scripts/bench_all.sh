#!/bin/bash
# the three bench lines (headline bandit with its CPU baseline, linear, darkroom)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_bandit.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload linear --no-cpu-baseline > gpurun_out/bench_linear.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload darkroom > gpurun_out/bench_darkroom.log 2>&1
timeout -k 10 600 python bench.py --workload darkroom --tasks 8192 > gpurun_out/bench_darkroom_c5.log 2>&1
