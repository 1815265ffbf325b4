#!/bin/bash
# GPU tests (incl. prefill parity) + smoke, then forward timing
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/gpu_tests.sh || exit $?
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || exit 1
timeout -k 10 600 python scripts/fwd_timing.py > gpurun_out/fwd_timing.log 2>&1
