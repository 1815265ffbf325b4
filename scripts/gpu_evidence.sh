#!/bin/bash
# end-of-round evidence on one box: GPU suite + smoke, the DarkRoom and bandit rocprofv3 passes, the
# bench line (headline + darkroom_c3 + CPU baselines) and the DarkRoom logit error, each step under
# its own time limit; stops at the first failure
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r5d}
bash scripts/gpu_tests.sh || exit $?
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || exit 1
bash scripts/profile_darkroom.sh $TAG || exit $?
bash scripts/profile_bandit.sh $TAG || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 200 python scripts/dr_logit_error.py > gpurun_out/logit_err_$TAG.json 2>&1
