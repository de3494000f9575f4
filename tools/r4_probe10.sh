#!/bin/bash
# Round-4 probe 10: down1.3 touching the next-but-one input window into L2 (UNET_MI355X_XSPF=1) --
# bitwise test, then two in-process interleaved A/Bs, mixed bs256.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v -k "window_prefetch" --timeout 200 \
  --timeout-method thread > gpurun_out/${TAG}_xspf_test.log 2>&1
echo "xspf test ok"
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 --cands "" "||UNET_MI355X_XSPF=1" \
    > gpurun_out/${TAG}_xspf_ab_$i.txt 2>&1
  echo "ab $i ok"
done
