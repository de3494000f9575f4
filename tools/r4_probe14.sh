#!/bin/bash
# Round-4 probe 14: x_to_px4 with a C == 3 fast path (three unconditional plane loads) against the previous
# build (libunet_mi355x_base.so), at bs256 and bs1, mixed; the pre-cast's per-launch time (slot 0, "down1.0").
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
D=tw-invoice-unet-ocr-llm_amd/unet_mi355x
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -q -k "golden_logits or u8_nhwc or reference_512 or masks_512_all" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
echo "tests ok"
for bs in 256 1; do
  for b in base new; do
    L=$D/libunet_mi355x.so; [ $b = base ] && L=$D/libunet_mi355x_base.so
    UNET_MI355X_LIB=$L timeout -k 10 200 python tools/tune.py --dtype mixed --batch $bs --reps 6 --cands "" > gpurun_out/${TAG}_bs${bs}_$b.txt 2>&1
  done
  echo "bs$bs ok"
done
