#!/bin/bash
# copy one gpu_round.sh pass (gpurun_out/) into profiles/<TAG>/ (run here, not on the box)
set -e
TAG=$1; G=gpurun_out; D=profiles/$TAG
mkdir -p $D
cp $G/prof_$TAG/trace/run_kernel_stats.csv $D/bandit_kernel_stats.csv
cp $G/prof_$TAG/pmc_fetch/run_counter_collection.csv $D/pmc_fetch_size.csv
cp $G/prof_$TAG/pmc_write/run_counter_collection.csv $D/pmc_write_size.csv
cp $G/prof_$TAG/pmc_l2/run_counter_collection.csv $D/pmc_tcc_hit_miss.csv
if [ -d $G/prof_dr_$TAG ]; then
  cp $G/prof_dr_$TAG/trace/run_kernel_stats.csv $D/darkroom_kernel_stats.csv
  cp $G/prof_dr_$TAG/pmc_mfma/run_counter_collection.csv $D/darkroom_pmc_mfma.csv
  cp $G/prof_dr_$TAG/pmc_mem/run_counter_collection.csv $D/darkroom_pmc_fetch.csv
fi
for w in bandit linear darkroom darkroom_c5; do
  [ -f $G/bench_$w.log ] && tail -n1 $G/bench_$w.log > $D/bench_$w.json
done
[ -f $G/gpu_tests.log ] && cp $G/gpu_tests.log $D/gpu_tests.log.txt
[ -f $G/smoke.log ] && cp $G/smoke.log $D/smoke.log.txt
ls $D
