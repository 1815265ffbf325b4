#!/bin/bash
# GPU tests (one process) then a library A/B at config 2 (AB_LIBS)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -n "$AB_LIBS" ]; then bash scripts/gpu_ab2.sh || exit $?; fi
