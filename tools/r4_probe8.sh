#!/bin/bash
# Round-4 probe 8: down2.0 (Cin = 64, Cout = 128; layer 1) on the 64-row weight-stationary ring
# (CFG_RING8_R64_WS = 10: all its weights resident, only the halo streams -- the conv1.3 kernel) and on
# the 9-tap 64-row ring (CFG_RING8_R64_T9 = 9) against the default 128-row 3-tap ring, in one process.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 --cands "" "1:10" "1:9" \
    > gpurun_out/${TAG}_d2a_cfgs_$i.txt 2>&1
  echo "cfgs $i ok"
done
