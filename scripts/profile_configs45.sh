#!/bin/bash
# rocprofv3 evidence for BASELINE configs 4 and 5 on one GPU (the per-GPU shards the bench line's
# linear_c4_shard / darkroom_c5_shard sub-objects time): kernel trace + stats of each, and the HBM
# PMC passes of the linear rollout (FETCH_SIZE, WRITE_SIZE, TCC hit/miss; one group per pass).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r6}
OUT=gpurun_out/prof45_$TAG
mkdir -p $OUT
LIN="bench.py --workload linear --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/lin_trace -o run -- \
    python3 $LIN --steps 2 --warmup 1 > $OUT/lin_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/lin_pmc_fetch -o run -- \
    python3 $LIN --steps 1 --warmup 0 > $OUT/lin_fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $OUT/lin_pmc_write -o run -- \
    python3 $LIN --steps 1 --warmup 0 > $OUT/lin_write.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T --output-format csv -d $OUT/lin_pmc_l2 -o run -- \
    python3 $LIN --steps 1 --warmup 0 > $OUT/lin_l2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/c5_trace -o run -- \
    python3 bench.py --workload darkroom --tasks 8192 --no-cpu-baseline --steps 1 --warmup 1 > $OUT/c5_trace.log 2>&1 || exit $?
find $OUT -name "*.csv" | sort > $OUT/files.txt
