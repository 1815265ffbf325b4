#!/bin/bash
# DarkRoom memo-hit chain on the whole tail wave (DPT_DR_HIT_WAVE): the DarkRoom tests, then A/B at
# config 3 and window 201 against the thread-0 chain (libdpt_hip_hit0.so)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -v -s -m gpu --timeout 400 \
    --timeout-method thread -k "darkroom" > gpurun_out/t7.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t7.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in 1 2; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=3 timeout -k 10 500 python scripts/ab_lib.py libdpt_hip_hit0.so libdpt_hip.so \
        > gpurun_out/ab7_R$R.json 2> gpurun_out/ab7_R$R.err || exit $?
done
