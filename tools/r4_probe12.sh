#!/bin/bash
# Round-4 probe 12: rocprofv3 kernel traces of the batch-1 forward (the app's call shape) at the mixed plan
# and at the drop-in default fp32, bench.py's step at N = 1 (the small-batch split-K plan), 30 steps each.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
P="--batch 1 --steps 30 --warmup 5 --no-cpu-baseline --no-latency --no-strong --no-fp32 --no-cfg5"
for dt in mixed fp32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_bs1_$dt -o run -- \
      python3 bench.py $P --dtype $dt > gpurun_out/prof_bench_${TAG}_bs1_$dt.json 2> gpurun_out/prof_${TAG}_bs1_$dt.err
  python tools/prof_summary.py gpurun_out/prof_${TAG}_bs1_$dt/run_kernel_trace.csv > gpurun_out/prof_${TAG}_bs1_$dt/summary.txt
  echo "bs1 $dt ok"
done
