#!/bin/bash
# the r6e evidence pass on the final build (dpt_darkroom.hip with the register-pressure trackers)
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_evidence.sh r6e
