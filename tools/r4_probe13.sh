#!/bin/bash
# Round-4 probe 13: 32-bit index math in the element kernels (x_to_px4, the fp32 first conv, the split-K
# reduction) -- the GPU suite, then the batch-1 per-launch times of the previous build
# (libunet_mi355x_base.so) and this one, mixed and fp32, 20 reps each.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
D=tw-invoice-unet-ocr-llm_amd/unet_mi355x
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.log 2>&1
echo "gpu tests ok"
for dt in mixed fp32; do
  for b in base new; do
    L=$D/libunet_mi355x.so; [ $b = base ] && L=$D/libunet_mi355x_base.so
    UNET_MI355X_LIB=$L timeout -k 10 200 python tools/tune.py --dtype $dt --batch 1 --reps 20 --cands "" > gpurun_out/${TAG}_bs1_${dt}_$b.txt 2>&1
  done
  echo "bs1 $dt ok"
done
