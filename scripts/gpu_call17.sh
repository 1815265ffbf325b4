#!/bin/bash
# DarkRoom C3 launch time against the task count (one workgroup per task, three per CU = 768 slots):
# how much of the 4096-task launch is the partly filled last round of workgroups
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
: > gpurun_out/dr_n_sweep.jsonl
for N in 768 1536 2304 3072 3840 4096 4352 4608; do
    AB_WL=darkroom AB_N=$N AB_DIGEST=0 AB_ROUNDS=1 timeout -k 10 300 python scripts/ab_lib.py libdpt_hip.so \
        > gpurun_out/dr_n_$N.json 2>> gpurun_out/dr_n_sweep.err || exit $?
    echo "{\"N\": $N, \"res\": $(grep -v amdgpu gpurun_out/dr_n_$N.json)}" >> gpurun_out/dr_n_sweep.jsonl
done
