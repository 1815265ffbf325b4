#!/bin/bash
# more hipcc scheduler options (on every file; dpt_darkroom keeps the trackers): DarkRoom config 3
# and the bandit rollout against the product build
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_WL=darkroom AB_DR_R=1 AB_ROUNDS=4 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_nounc.so \
    libdpt_hip_relax.so libdpt_hip_mb0.so libdpt_hip_vgprf.so > gpurun_out/ab21_R1.json 2> gpurun_out/ab21_R1.err || exit $?
AB_ROUNDS=4 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_nounc.so libdpt_hip_relax.so \
    libdpt_hip_mb0.so libdpt_hip_vgprf.so > gpurun_out/ab21_bandit.json 2> gpurun_out/ab21_bandit.err
