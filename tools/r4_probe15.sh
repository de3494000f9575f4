#!/bin/bash
# Round-4 probe 15: the fp32 first conv with its weights through scalar loads (no LDS staging) -- fp32 tests,
# then per-launch times of the previous build (libunet_mi355x_base.so) and this one, fp32 at bs1 and bs32.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
D=tw-invoice-unet-ocr-llm_amd/unet_mi355x
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -q -k "golden or odd_shapes or nan or reference_512 or minimum_size or fp32" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "tests ok"
for bs in 1 32; do
  for b in base new; do
    L=$D/libunet_mi355x.so; [ $b = base ] && L=$D/libunet_mi355x_base.so
    UNET_MI355X_LIB=$L timeout -k 10 200 python tools/tune.py --dtype fp32 --batch $bs --reps 10 --cands "" > gpurun_out/${TAG}_fp32_bs${bs}_$b.txt 2>&1
  done
  echo "bs$bs ok"
done
