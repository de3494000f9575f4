#!/bin/bash
# Round-4 probe 5: per-layer static wave priority (UNET_MI355X_PRIO_LAYERS) on the layers where the
# global option helped in tune_r4c_setprio_neutral.txt (down1.3, down2.0, conv1.3, up4, up3), two
# in-process interleaved runs of the experimental build.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
L=tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x_exp.so
for i in 1 2; do
  UNET_MI355X_LIB=$L timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 --cands "" "||UNET_MI355X_PRIO_LAYERS=0,1,16,17,18" "||UNET_MI355X_PRIO=1" > gpurun_out/${TAG}_prio_layers_$i.txt 2>&1
  echo "prio $i ok"
done
