#!/bin/bash
# quick kernel iteration: the kernel parity tests of one workload (AB_TESTS, a pytest -k
# expression), then an A/B of library builds (AB_LIBS; AB_WL=darkroom for config 3)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread -k "${AB_TESTS:-darkroom}" > gpurun_out/t_quick.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t_quick.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python scripts/ab_lib.py ${AB_LIBS:-libdpt_hip.so} > gpurun_out/ab.log 2>&1
