#!/bin/bash
# hipcc scheduler strategies on the DarkRoom kernel: max-ilp, max-memory-clause and the AMDGPU
# register-pressure trackers against the default build, config 3 (digests: bit-identity)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_WL=darkroom AB_DR_R=1 AB_ROUNDS=3 timeout -k 10 600 python scripts/ab_lib.py libdpt_hip.so libdpt_hip_ilp.so \
    libdpt_hip_memcl.so libdpt_hip_trk.so > gpurun_out/ab18.json 2> gpurun_out/ab18.err
