#!/bin/bash
# GPU suite, then an A/B of library builds (AB_LIBS; AB_WL=darkroom for config 3, else the
# bandit at AB_H/AB_N/AB_A) and the DarkRoom logit error against the reference fixtures
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python scripts/ab_lib.py ${AB_LIBS:-libdpt_hip.so} > gpurun_out/ab.log 2>&1 || exit $?
timeout -k 10 200 python scripts/dr_logit_error.py > gpurun_out/logit_err.log 2>&1
