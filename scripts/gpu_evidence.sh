#!/bin/bash
# end-of-round evidence on one box: build provenance, GPU suite + smoke, the DarkRoom and bandit
# rocprofv3 passes, the bench line (headline + darkroom_c3 / darkroom_c5_shard / linear_c4_shard
# + CPU baselines) and the DarkRoom logit error, each step under its own time limit; stops at the
# first failure
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-r6}
LIB=decision-pretrained-transformer_amd/dpt_hip/libdpt_hip.so
# build provenance: the pushed library (the one every step below loads) was linked from the sources
# whose hash the Makefile recorded next to it (libdpt_hip.so.srchash); the same hash of the pushed
# sources on the box means the evidence runs the HEAD build, without rebuilding it
CSRC=decision-pretrained-transformer_amd/csrc
{
    echo "library_sha256 $(sha256sum $LIB | cut -d' ' -f1)"
    echo "library_built_from $(cat $LIB.srchash 2>/dev/null || echo missing)"
    now=$(cd $CSRC && cat dpt_abi.hip dpt_decode.hip dpt_env.hip dpt_policies.hip dpt_darkroom.hip dpt_prefill.hip \
          dpt_stats.hip dpt_train.hip dpt_common.h dpt_mfma_fwd.h dpt_linucb.h ../../include/dpt_hip.h Makefile | sha256sum | cut -d' ' -f1)
    echo "pushed_sources $now"
    if [ "$now" = "$(cat $LIB.srchash 2>/dev/null)" ]; then echo "library matches the pushed sources: yes"
    else echo "library matches the pushed sources: NO"; fi
    echo "hipcc $(/opt/rocm/bin/hipcc --version 2>/dev/null | grep -m1 -i 'clang version')"
} > gpurun_out/provenance_$TAG.txt 2>&1
grep -q "matches the pushed sources: yes" gpurun_out/provenance_$TAG.txt || exit 1
bash scripts/gpu_tests.sh || exit $?
grep -q "pytest rc=0" gpurun_out/gpu_tests.log || exit 1
bash scripts/profile_darkroom.sh $TAG || exit $?
bash scripts/profile_bandit.sh $TAG || exit $?
bash scripts/profile_configs45.sh $TAG || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 200 python scripts/dr_logit_error.py > gpurun_out/logit_err_$TAG.json 2>&1
