#!/bin/bash
# full evidence pass: GPU tests + smoke, profiles of both kernels, bench lines
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r1}
bash scripts/gpu_tests.sh || exit $?
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || exit 1
bash scripts/profile_bandit.sh $TAG || exit $?
bash scripts/profile_darkroom.sh $TAG || exit $?
bash scripts/bench_all.sh
