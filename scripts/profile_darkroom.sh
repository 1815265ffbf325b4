#!/bin/bash
# rocprofv3 evidence for the fused DarkRoom kernel (config 3): kernel trace + stats, then
# separate PMC passes (one counter group per pass, each under its own time limit):
#  mfma   SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (matrix-pipe busy fraction, effective clock)
#  mem    FETCH_SIZE (HBM bytes; x2 on gfx950)
#  stall  where the wave cycles go (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_*)
#  insts  instruction mix (VALU, MFMA, LDS, SALU, transcendental, cvt, fp64)
#  lds    LDS bank conflicts / LDS-issue stalls / VALU-MFMA co-execution
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r1}
OUT=gpurun_out/prof_dr_$TAG
mkdir -p $OUT
BENCH="bench.py --workload darkroom --no-cpu-baseline"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/trace -o run -- \
    python3 $BENCH --steps 2 --warmup 1 > $OUT/bench_trace.log 2>&1 || exit $?
pass() {
    local name=$1; shift
    timeout -s KILL 300 rocprofv3 --pmc "$@" -T --output-format csv -d $OUT/pmc_$name -o run -- \
        python3 $BENCH --steps 1 --warmup 0 > $OUT/bench_$name.log 2>&1
}
pass mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
pass mem FETCH_SIZE || exit $?
pass stall SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC || exit $?
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_SMEM || exit $?
pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_BRANCH || exit $?
find $OUT -name "*.csv" | sort > $OUT/files.txt
