#!/bin/bash
# round-6 first GPU pass: the DarkRoom / full-config parity tests, then the workspace-free bisect
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_dropin.py tests/test_gpu_train.py -v -s -m gpu --timeout 400 --timeout-method thread \
    -k "darkroom or full_config or policy or dropout or baseline or linucb" > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/t1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -u scripts/dr_nows_bisect.py scratch/nows/19939cb scratch/nows/7d8530e scratch/nows/0fcb079 \
    scratch/nows/a79aebc scratch/nows/1111a25 scratch/nows/3c9b0eb scratch/nows/6bfd96c scratch/nows/84d7166 . \
    .:libdpt_hip_nows0.so > gpurun_out/bisect.jsonl 2> gpurun_out/bisect.err
