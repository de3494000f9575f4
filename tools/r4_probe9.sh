#!/bin/bash
# Round-4 probe 9: the short-K layers (down2.0, down3.0, down4.0: a tile epilogue every 6-24 steps) on the
# 4-wave 128-row ring with two blocks per CU (CFG_RING_R128 = 3: the second block's MFMAs cover one
# block's epilogue), and conv1.0 on the 4-wave 64-row 3-tap ring (CFG_RING_R64_T3 = 4), in one process.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 --cands "" "1:3,3:3,5:3" "15:4" \
    > gpurun_out/${TAG}_shortk_cfgs_$i.txt 2>&1
  echo "cfgs $i ok"
done
