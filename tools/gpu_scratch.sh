#!/bin/bash
# scratch GPU pass (edited per call)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread \
    -k "fp32 or labels or small_batch or split or head or mask" > gpurun_out/gpu_tests_r6t.log 2>&1
echo tests ok
timeout -k 10 200 python tools/tune.py --dtype fp32 --batch 32 --reps 3 --cands "" > gpurun_out/tune_bs32_r6t.txt 2>&1
timeout -k 10 200 python tools/tune.py --dtype fp32 --batch 1 --reps 7 --cands "" > gpurun_out/tune_bs1_r6t.txt 2>&1
echo tune ok
