#!/bin/bash
# Round-4 probes, third set: the GPU tests on the current library, then batch-1 per-layer times of the
# current library (64-row split slices) against the previous build (libunet_mi355x_base.so), fp32 and
# mixed, and the bench line.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
echo "tests ok"
D=tw-invoice-unet-ocr-llm_amd/unet_mi355x
for dt in mixed fp32; do
  for b in base new; do
    L=$D/libunet_mi355x.so; [ $b = base ] && L=$D/libunet_mi355x_base.so
    UNET_MI355X_LIB=$L timeout -k 10 200 python tools/tune.py --dtype $dt --batch 1 --reps 30 --cands "" > gpurun_out/${TAG}_bs1_${dt}_$b.txt 2>&1
  done
done
echo "bs1 ok"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench ok"
