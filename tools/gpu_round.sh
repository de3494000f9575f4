#!/bin/bash
# One GPU-box pass: gpu tests, default bench line, rocprofv3 kernel stats, PMC HBM passes.
# Usage (from this container): gpurun --timeout 1200 -- 'bash tools/gpu_round.sh TAG'
set -e
TAG=${1:-r1}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
echo tests ok
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
timeout -k 10 300 python bench.py --size 1024 --batch 64 --dtype fp16 --steps 3 --cpu-seconds 10 > gpurun_out/bench_${TAG}_cfg5_fp16_1024.json 2> gpurun_out/bench_${TAG}_cfg5.err
echo bench cfg5 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err
echo prof ok
mkdir -p gpurun_out/pmc_$TAG
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d gpurun_out/pmc_$TAG/pass_$c -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-layer-profile > gpurun_out/pmc_$TAG/$c.log 2>&1
done
echo pmc ok
python tools/pmc_summary.py gpurun_out/pmc_$TAG --bench-json gpurun_out/prof_bench_$TAG.json --out gpurun_out/pmc_$TAG/summary.json > gpurun_out/pmc_$TAG/summary.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --min-grid 10000 > gpurun_out/prof_$TAG/summary.txt
echo summaries ok
