#!/bin/bash
# DarkRoom parity over the whole population of config 3 and of config 5's first shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/dr_full_population.py > gpurun_out/dr_full_population.jsonl \
    2> gpurun_out/dr_full_population.err
