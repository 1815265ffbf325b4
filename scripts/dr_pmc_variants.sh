#!/bin/bash
# instruction counts of the DarkRoom kernel per library build (timing-only variants that leave phases out:
# the differences attribute the VALU / SALU / MFMA / LDS instructions to the phases)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/drpmc
export TMPDIR=/tmp
for lib in "$@"; do
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 \
        SQ_INSTS_VALU_CVT -T --output-format csv -d gpurun_out/drpmc/$lib -o run -- python3 scripts/dr_pmc_run.py $lib \
        > gpurun_out/drpmc/$lib.log 2>&1 || exit $?
done
