#!/bin/bash
# Stochastic PC sampling (rocprofv3, gfx950) of the fused DarkRoom kernel: which instructions the
# waves sit on, with the stall reason.  Lists the available sampling configurations first.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1 || exit $?
grep -i -A12 "pc.sampl" gpurun_out/pcs/list.txt | head -60 > gpurun_out/pcs/pc_configs.txt
METHOD=${PCS_METHOD:-stochastic}
UNIT=${PCS_UNIT:-cycles}
INTERVAL=${PCS_INTERVAL:-65536}
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
    --pc-sampling-interval $INTERVAL --kernel-trace --output-format csv -d gpurun_out/pcs/run -o pcs -- \
    python3 scripts/dr_pc_run.py > gpurun_out/pcs/run.log 2>&1
echo "rc=$?" >> gpurun_out/pcs/run.log
