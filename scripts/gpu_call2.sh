#!/bin/bash
# round-6 second GPU pass: LinUCB / dropout tests, bench line with the config-4/5 sub-objects,
# PC sampling of the DarkRoom kernel
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_train.py -v -s -m gpu --timeout 300 \
    --timeout-method thread -k "linucb or dropout or policy" > gpurun_out/t2.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t2.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench2.json 2> gpurun_out/bench2.err || exit $?
bash scripts/pc_sample_darkroom.sh
