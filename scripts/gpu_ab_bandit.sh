#!/bin/bash
# GPU suite, then a bandit A/B of library builds (AB_LIBS, config 2; AB_H / AB_A for others)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_ROUNDS=3 timeout -k 10 400 python scripts/ab_lib.py ${AB_LIBS:-libdpt_hip.so} > gpurun_out/ab.log 2>&1 || exit $?
AB_ROUNDS=2 AB_H=1000 AB_A=20 timeout -k 10 400 python scripts/ab_lib.py ${AB_LIBS:-libdpt_hip.so} > gpurun_out/ab_linear.log 2>&1
