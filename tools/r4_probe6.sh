#!/bin/bash
# Round-4 probe 6: where the 3-tap 128-row ring's time goes -- timing-only ablations of
# conv3x3_ring8_kernel on the 13 layers that run it (d2a .. c2a; c2b carries the fused up1), in one
# process, interleaved: 1 = no barriers, 2 = no MFMAs, 3 = no LDS fragment reads, 4 = no LDS-DMA
# in the loop (libunet_mi355x_abl.so; cfg = CFG_RING8_R128 + 16 * ablation; wrong outputs by construction).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
L=tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x_abl.so
c() { local v=$1 s=""; for i in 1 2 3 4 5 6 7 8 9 10 11 12 13; do s="$s${s:+,}$i:$v"; done; echo "$s"; }
UNET_MI355X_LIB=$L timeout -k 10 400 python tools/tune.py --dtype mixed --batch 256 --reps 3 \
  --cands "" "$(c 24)" "$(c 40)" "$(c 56)" "$(c 72)" > gpurun_out/${TAG}_ring8_ablation.txt 2>&1
echo "ablation ok"
