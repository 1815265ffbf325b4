#!/bin/bash
# list gfx950 counters, then a few SQ stall / LDS counters on the DarkRoom kernel (one group per pass)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/probe; export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/probe/counters.txt 2>&1
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_WAIT_ANY SQ_ACTIVE_INST_MISC"; do
  tag=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp -T --output-format csv -d gpurun_out/probe/$tag -o run -- \
      python3 scripts/dr_once.py > gpurun_out/probe/$tag.log 2>&1 || echo "FAILED $grp" >> gpurun_out/probe/failed.txt
done
