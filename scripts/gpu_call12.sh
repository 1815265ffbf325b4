#!/bin/bash
# branch-free masked score tiles (the MFMA hazard fix) with the first-pair peel: the DarkRoom tests on
# the product build, then A/B at config 3 and window 201 against HEAD (libdpt_hip_head.so), the fixed
# build without the peel (nopeel) and with the unrolled pair loop (unroll)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py -v -s -m gpu --timeout 400 \
    --timeout-method thread -k "darkroom" > gpurun_out/t12.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t12.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for R in 1 2; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=3 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip_head.so libdpt_hip_nopeel.so \
        libdpt_hip.so libdpt_hip_unroll.so > gpurun_out/ab12_R$R.json 2> gpurun_out/ab12_R$R.err || exit $?
done
