#!/bin/bash
# scheduler strategies, second pass: max-ilp, the register-pressure trackers and both, against the
# default build at config 3, window 201 and on the bandit rollout (the flags apply to the library)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in 1 2; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=5 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_ilp.so \
        libdpt_hip_trk.so libdpt_hip_ilptrk.so > gpurun_out/ab19_R$R.json 2> gpurun_out/ab19_R$R.err || exit $?
done
AB_ROUNDS=3 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_ilp.so libdpt_hip_trk.so \
    libdpt_hip_ilptrk.so > gpurun_out/ab19_bandit.json 2> gpurun_out/ab19_bandit.err
