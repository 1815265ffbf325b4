#!/bin/bash
# round-6 third GPU pass: the long-window DarkRoom kernels with one block at a time (kSeqBlocks):
# tests, then A/B at windows 101 / 201 / 301 against the base build and the DPT_DR_SEQ_BLOCKS=0
# build, then per-phase stamps of the config-3 kernel (memo off / on)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -v -s -m gpu --timeout 300 --timeout-method thread \
    -k "long_windows or windows_over_256 or workspace_free or dim12 or memo_bit or darkroom_fused or philox_vs_oracle" \
    > gpurun_out/t3.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/t3.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
AB_WL=darkroom AB_DR_R=1 AB_ROUNDS=3 timeout -k 10 400 python scripts/ab_lib.py libdpt_hip_r6base.so libdpt_hip.so \
    libdpt_hip_short8.so > gpurun_out/ab3_R1.json 2> gpurun_out/ab3_R1.err || exit $?
for R in 2 3; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=3 timeout -k 10 400 python scripts/ab_lib.py libdpt_hip_r6base.so libdpt_hip.so \
        libdpt_hip_seq0.so > gpurun_out/ab3_R$R.json 2> gpurun_out/ab3_R$R.err || exit $?
done
DR_MEMO=0 timeout -k 10 300 python scripts/dr_stamps.py > gpurun_out/stamps_memo0.json 2>&1 || exit $?
DR_MEMO=1 timeout -k 10 300 python scripts/dr_stamps.py > gpurun_out/stamps_memo1.json 2>&1
