#!/bin/bash
# the register-pressure trackers on dpt_darkroom.hip only (product build) against the same sources
# without them (libdpt_hip_notrk.so): DarkRoom tests, then windows 101 / 201 / 301
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -v -s -m gpu --timeout 400 \
    --timeout-method thread -k "darkroom" > gpurun_out/t20.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t20.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in 1 2 3; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=4 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip_notrk.so libdpt_hip.so \
        > gpurun_out/ab20_R$R.json 2> gpurun_out/ab20_R$R.err || exit $?
done
