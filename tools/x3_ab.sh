#!/bin/bash
# fp32 plan: three bf16 terms (the default, UNET_DTYPE_F32) vs the exact-fp32 MFMA (UNET_MI355X_F32X3=0 =
# UNET_DTYPE_F32_EXACT's kernels) -- per-layer A/B timing at the config-2 shape (batch 32, 512^2) and batch 1.
# Usage: gpurun -- "bash tools/x3_ab.sh TAG"
set -e
TAG=${1:-x3}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune.py --dtype fp32 --batch 32 --reps 3 --cands "" "||UNET_MI355X_F32X3=0" \
    > gpurun_out/x3_tune_$TAG.txt 2>&1
timeout -k 10 300 python tools/tune.py --dtype fp32 --batch 1 --reps 5 --cands "" "||UNET_MI355X_F32X3=0" \
    > gpurun_out/x3_tune_bs1_$TAG.txt 2>&1
echo tune ok
