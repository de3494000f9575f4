#!/bin/bash
# After `gpurun -- "bash tools/gpu_round.sh TAG COMMIT"`: copy the call's outputs that are judged into
# profiles/ (tracked) -- rocprof kernel stats + summaries, PMC summaries (and the bench's traffic sources),
# the driver-shaped bench lines, the stamp and the GPU test log.  Usage: bash tools/copy_round_profiles.sh TAG
set -e
T=$1
G=gpurun_out
P=profiles
for leg in ":mixed_bs256:pmc_mixed_bs256.json" "_cfg5:cfg5_fp16_1024_bs64:pmc_fp16_bs64_1024.json" "_fp32:fp32_bs32:pmc_fp32_bs32.json"; do
  IFS=: read -r suf name tj <<< "$leg"
  cp $G/prof_$T$suf/run_kernel_stats.csv $P/rocprof_${T}_${name}_kernel_stats.csv
  cp $G/prof_$T$suf/summary.txt $P/rocprof_${T}_${name}_summary.txt
  cp $G/pmc_$T$suf/summary.txt $P/pmc_${T}_${name}_summary.txt
  cp $G/pmc_$T$suf/summary.json $P/$tj
done
cp $G/bench_$T.json $P/bench_${T}_mixed.json
cp $G/bench_$T.detail.json $P/bench_${T}_mixed.detail.json
cp $G/bench_${T}_cfg5_fp16_1024.json $P/bench_${T}_cfg5_fp16_1024_bs64.json
cp $G/stamp_$T.json $P/stamp_$T.json
cp $G/gpu_tests_$T.log $P/gpu_tests_$T.txt
cp $G/smoke_$T.log $P/smoke_$T.txt
echo copied
