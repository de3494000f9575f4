#!/bin/bash
# One GPU-box pass: GPU tests + smoke, then the driver-shaped bench line.
# Usage: gpurun --timeout 1200 -- "bash tools/gpu_check.sh TAG [skip-tests|tests-only] [pytest -k expr]"
set -e
TAG=${1:-r6}
MODE=${2:-}
K=${3:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$MODE" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread ${K:+-k "$K"} \
      > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo smoke ok
fi
[ "$MODE" = "tests-only" ] && exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail-out gpurun_out/bench_$TAG.detail.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
