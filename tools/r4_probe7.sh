#!/bin/bash
# Round-4 probe 7: the staggered 3-tap 128-row ring (UNET_MI355X_STAGGER on d2a .. c2a) -- bitwise test,
# then an in-process A/B against the default ring and against the previous default of no per-layer
# priority (UNET_MI355X_PRIO_LAYERS empty), two interleaved runs, mixed bs256.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v -k "staggered or deterministic" --timeout 150 \
  --timeout-method thread > gpurun_out/${TAG}_stagger_tests.log 2>&1
echo "stagger tests ok"
S=$(seq -s, 1 13)
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 \
    --cands "" "||UNET_MI355X_STAGGER=$S" "||UNET_MI355X_PRIO_LAYERS=" > gpurun_out/${TAG}_stagger_ab_$i.txt 2>&1
  echo "ab $i ok"
done
