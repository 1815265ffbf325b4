#!/bin/bash
# first GPU pass: kernel parity tests, smoke, short bench
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
rocminfo | grep -m3 -E "Marketing Name|gfx" > gpurun_out/rocminfo.txt 2>&1
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> gpurun_out/smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1
echo "bench rc=$?" >> gpurun_out/bench1.log
