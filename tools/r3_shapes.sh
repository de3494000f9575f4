#!/bin/bash
# Round-3 shapes pass: the per-rank strong-scaling shapes (N=32, N=128 per GPU: global batch 256
# and 1024 over 8 GPUs) and the fp32 config-2 leg (bs32, 512^2), each a bench line + a rocprofv3
# kernel-stats summary; then the default bench line (strong + fp32 legs + latency inside).
# Usage: gpurun --timeout 900 -- 'bash tools/r3_shapes.sh TAG [tests]'
set -e
TAG=${1:-r3a}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$2" == "tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
fi
P="--no-cpu-baseline --no-latency --no-strong --no-fp32"
for cfg in "fp32 32" "mixed 32" "mixed 128"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --dtype $1 --batch $2 --steps 20 --warmup 5 $P \
      > gpurun_out/bench_${TAG}_$1_bs$2.json 2> gpurun_out/bench_${TAG}_$1_bs$2.err
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$1_bs$2 -o run -- \
      python3 bench.py --dtype $1 --batch $2 --steps 5 --warmup 2 $P \
      > gpurun_out/prof_${TAG}_$1_bs$2.json 2> gpurun_out/prof_${TAG}_$1_bs$2.err
  python tools/prof_summary.py gpurun_out/prof_${TAG}_$1_bs$2/run_kernel_trace.csv --min-grid 100 > gpurun_out/prof_${TAG}_$1_bs$2/summary.txt
  echo $1 $2 ok
done
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_${TAG}.json 2> gpurun_out/bench_${TAG}.err
echo bench ok
