#!/bin/bash
# DarkRoom parity on every task of long-window batches (windows 201 / 301, workspace-free dim 12)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/dr_full_population.py --long > gpurun_out/dr_full_population_long.jsonl \
    2> gpurun_out/dr_full_population_long.err
