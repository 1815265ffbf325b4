#!/bin/bash
# rocprofv3 evidence for the fused DarkRoom kernel (config 3): kernel trace +
# stats, then separate PMC passes (MFMA busy cycles + GPU-active cycles for the
# effective clock; HBM FETCH/WRITE to show it is not memory-bound).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_dr_$TAG
mkdir -p $OUT
BENCH="bench.py --workload darkroom"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $BENCH --steps 2 --warmup 1 > $OUT/bench_trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -T --output-format csv -d $OUT/pmc_mfma -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_mfma.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $OUT/pmc_mem -o run -- \
    python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_mem.log 2>&1 || exit $?
find $OUT -name "*.csv" | sort > $OUT/files.txt
