#!/bin/bash
# bandit kernel iteration: kernel parity, tile A/B timing, FETCH_SIZE + L2 hit pass
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_kernels.py -x -q -m gpu > gpurun_out/t_kern.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/t_kern.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python scripts/ab_tile.py > gpurun_out/ab_tile.log 2>&1 || exit $?
rm -rf gpurun_out/bi_fetch gpurun_out/bi_l2
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d gpurun_out/bi_fetch -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/bi_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d gpurun_out/bi_l2 -o run -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/bi_l2.log 2>&1
