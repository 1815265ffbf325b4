#!/bin/bash
# tests -> full bench line -> rocprofv3 trace + PMC passes of the headline kernel
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
bash scripts/profile_bandit.sh ${TAG:-r1e}
