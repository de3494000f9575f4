#!/bin/bash
# Round-4 probes on one GPU box (after the GPU tests): batch-1 split-K on/off (fp32, mixed) and the
# XCD-owned row tiles A/B at the bench shape, in-process interleaved (tools/tune.py).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
for dt in mixed fp32; do
  timeout -k 10 200 python tools/tune.py --dtype $dt --batch 1 --reps 20 --cands "" "||UNET_MI355X_KSPLIT=0" > gpurun_out/${TAG}_bs1_ksplit_$dt.txt 2>&1
  echo "bs1 $dt ok"
done
timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 --cands "" "||UNET_MI355X_XCDROWS=8" "||UNET_MI355X_XCDROWS=5,6,7,8,9,10" > gpurun_out/${TAG}_xcdrows.txt 2>&1
echo "xcdrows ok"
