#!/bin/bash
# GPU tests, then DarkRoom bench with and without the per-episode logits memo.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload darkroom --steps 3 --warmup 1 > gpurun_out/bench_dr_memo.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload darkroom --steps 2 --warmup 1 --darkroom-memo 0 \
    > gpurun_out/bench_dr_nomemo.log 2>&1 || exit $?
