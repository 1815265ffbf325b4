#!/bin/bash
# the three bench lines (headline bandit with its CPU baseline, linear, darkroom)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench_bandit.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload linear --no-cpu-baseline > gpurun_out/bench_linear.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload darkroom > gpurun_out/bench_darkroom.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload darkroom --tasks 8192 > gpurun_out/bench_darkroom_c5.log 2>&1 || exit $?
timeout -k 10 300 python scripts/train_timing.py > gpurun_out/train_timing.json 2> gpurun_out/train_timing.err || exit $?
timeout -k 10 300 python scripts/dr_step_timing.py > gpurun_out/dr_step_timing.json 2> gpurun_out/dr_step_timing.err
