#!/bin/bash
# the headline kernel's trace + PMC again (profile_bandit.sh now excludes the linear sub-object,
# whose launches share the kernel name), and the two-rank bench test with the sub-objects
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/profile_bandit.sh r6a || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py -v -s -m gpu --timeout 600 --timeout-method thread \
    > gpurun_out/t5.log 2>&1
echo "pytest rc=$?" >> gpurun_out/t5.log
