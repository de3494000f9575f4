#!/bin/bash
# Round-4 probe 11: up2 on the 256-row x 128-pixel weight-stationary ConvTranspose (UNET_MI355X_CONVT_WS=2) --
# bitwise test, then two in-process interleaved A/Bs against the ring, mixed bs256.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v -k "weight_stationary_matches_ring or deterministic" \
  --timeout 200 --timeout-method thread > gpurun_out/${TAG}_ws2_tests.log 2>&1
echo "ws2 tests ok"
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 4 --cands "" "||UNET_MI355X_CONVT_WS=2" \
    > gpurun_out/${TAG}_ws2_ab_$i.txt 2>&1
  echo "ab $i ok"
done
