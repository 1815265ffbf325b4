#!/bin/bash
# full evidence pass: GPU tests + smoke, profiles of both kernels, bench lines
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r1}
bash scripts/gpu_tests.sh || exit $?
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || exit 1
bash scripts/profile_bandit.sh $TAG || exit $?
bash scripts/profile_darkroom.sh $TAG || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_bandit.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload linear --no-cpu-baseline > gpurun_out/bench_linear.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload darkroom > gpurun_out/bench_darkroom.log 2>&1
