#!/bin/bash
# bisect of the attend first-pair peel (DPT_ATT_PEEL 1..4, DPT_ATT_RFL): DarkRoom checksums and
# times against the unpeeled build (libdpt_hip_nopeel.so) at config 3 and window 201
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for R in 1 2; do
    AB_WL=darkroom AB_DR_R=$R AB_ROUNDS=1 timeout -k 10 400 python scripts/ab_lib.py libdpt_hip_nopeel.so libdpt_hip.so \
        libdpt_hip_p2.so libdpt_hip_p3.so libdpt_hip_p4.so libdpt_hip_rfl.so > gpurun_out/ab11_R$R.json 2> gpurun_out/ab11_R$R.err || exit $?
done
