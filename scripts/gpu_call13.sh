#!/bin/bash
# the r6d evidence pass on the code with the MFMA wait-state fix
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_evidence.sh r6d
