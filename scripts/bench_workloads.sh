#!/bin/bash
# secondary workloads: linear (config 4 shard) and darkroom (config 3)
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --workload linear --steps 1 --warmup 1 > gpurun_out/bench_linear.log 2>&1 || exit $?
timeout -k 10 900 python bench.py --workload darkroom --steps 1 --warmup 0 > gpurun_out/bench_darkroom.log 2>&1 || exit $?
