#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/h_sweep.py > gpurun_out/h_sweep.log 2>&1
