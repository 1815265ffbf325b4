#!/bin/bash
# GPU test pass: pytest -m gpu (one process, per-test timeout), then smoke.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.log
exit $rc
