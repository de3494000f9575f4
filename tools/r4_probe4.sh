#!/bin/bash
# Round-4 probes, fourth set: GPU tests, batch-1 per-layer times against the previous build
# (libunet_mi355x_base.so), the weight-stationary ConvTranspose A/B at the bench shape, the bench line.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
echo "tests ok"
D=tw-invoice-unet-ocr-llm_amd/unet_mi355x
for b in base new; do
  L=$D/libunet_mi355x.so; [ $b = base ] && L=$D/libunet_mi355x_base.so
  UNET_MI355X_LIB=$L timeout -k 10 200 python tools/tune.py --dtype mixed --batch 1 --reps 30 --cands "" > gpurun_out/${TAG}_bs1_mixed_$b.txt 2>&1
done
echo "bs1 ok"
timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 --cands "" "||UNET_MI355X_CONVT_WS=0" > gpurun_out/${TAG}_convt_ws.txt 2>&1
echo "ws ok"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo "bench ok"
