#!/bin/bash
# rocprofv3 evidence for the headline kernel (run on the GPU box via gpurun).
#  1. kernel trace + stats of the bench command (durations, per-kernel summary)
#  2. separate PMC passes: FETCH_SIZE, then WRITE_SIZE (TCC slots: 3 + 2 > 4)
# Outputs under gpurun_out/prof_<tag>/ ; copy the summaries into profiles/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
BENCH="bench.py --no-cpu-baseline --no-darkroom --no-linear"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $BENCH --steps 3 --warmup 1 > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_fetch -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/pmc_write -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d $OUT/pmc_l2 -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_l2.log 2>&1 || exit $?
find $OUT -name "*.csv" | sort > $OUT/files.txt
