#!/bin/bash
# DarkRoom parity on every task of config 3, greedy and with permuted actions
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u scripts/dr_full_population.py --variants > gpurun_out/dr_full_population_variants.jsonl \
    2> gpurun_out/dr_full_population_variants.err
