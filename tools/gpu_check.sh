#!/bin/bash
# One GPU-box pass without profiles: GPU tests + smoke, the driver-shaped bench line, and the same
# headline at world size 1 through the N > 1 code path (bench.py --dist: nccl process group, RCCL
# all-gather inside the step, device MAX all-reduce) for the "within 1 %" comparison.
# Usage: gpurun --timeout 1200 -- "bash tools/gpu_check.sh TAG [skip-tests|tests-only]"
set -e
TAG=${1:-r5}
MODE=${2:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$MODE" != "skip-tests" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo smoke ok
fi
[ "$MODE" = "tests-only" ] && exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail-out gpurun_out/bench_$TAG.detail.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
P="--no-cpu-baseline --no-latency --no-fp32 --no-cfg5 --no-strong"
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 $P --detail-out gpurun_out/bench_${TAG}_plain$i.detail.json \
      > gpurun_out/bench_${TAG}_plain$i.json 2> gpurun_out/bench_${TAG}_plain$i.err
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --dist $P --detail-out gpurun_out/bench_${TAG}_dist$i.detail.json \
      > gpurun_out/bench_${TAG}_dist$i.json 2> gpurun_out/bench_${TAG}_dist$i.err
done
echo dist ok
