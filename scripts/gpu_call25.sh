#!/bin/bash
# DarkRoom parity on every task of config 5's last shard
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/dr_full_population.py --lastshard > gpurun_out/dr_full_population_lastshard.jsonl \
    2> gpurun_out/dr_full_population_lastshard.err
