#!/bin/bash
# Copy one tools/gpu_round.sh pass (gpurun_out/, tag TAG) into profiles/ under the tracked names.
# Usage: bash tools/copy_round_profiles.sh TAG
set -e
T=$1; G=gpurun_out; P=profiles
cp $G/bench_$T.json $P/bench_${T}_mixed.json
cp $G/bench_$T.detail.json $P/bench_${T}_mixed.detail.json
cp $G/bench_${T}_cfg5_fp16_1024.json $P/bench_${T}_cfg5_fp16_1024_bs64.json
cp $G/gpu_tests_$T.log $G/smoke_$T.log $G/stamp_$T.json $P/
cp $G/pmc_$T/summary.txt $P/pmc_${T}_mixed_bs256_summary.txt
cp $G/pmc_${T}_cfg5/summary.txt $P/pmc_${T}_cfg5_fp16_1024_bs64_summary.txt
cp $G/pmc_${T}_fp32/summary.txt $P/pmc_${T}_fp32_bs32_summary.txt
# the bench's traffic sources (bench.py reads these; stamped with the kernel sources' hash)
cp $G/pmc_$T/summary.json $P/pmc_mixed_bs256.json
cp $G/pmc_${T}_cfg5/summary.json $P/pmc_fp16_bs64_1024.json
cp $G/pmc_${T}_fp32/summary.json $P/pmc_fp32_bs32.json
for S in "" _cfg5 _fp32; do
  case "$S" in "") N=mixed_bs256;; _cfg5) N=cfg5_fp16_1024_bs64;; _fp32) N=fp32_bs32;; esac
  cp $G/prof_$T$S/run_kernel_stats.csv $P/rocprof_${T}_${N}_kernel_stats.csv
  cp $G/prof_$T$S/summary.txt $P/rocprof_${T}_${N}_summary.txt
done
python3 tools/pmc_clock.py $G/pmc_$T > $P/pmc_${T}_clock_mfma_waits.txt
