#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python scripts/phase_stamps.py > gpurun_out/stamps.log 2>&1
