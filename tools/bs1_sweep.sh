#!/bin/bash
# Batch-1 split-K sweep of a precision plan: every eligible layer forced to each slice count (and the automatic
# plan), per-layer times side by side (tools/tune.py).  Usage: gpurun -- "bash tools/bs1_sweep.sh TAG DTYPE"
set -e
TAG=$1; DT=${2:-fp32}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
force() { local s=""; for i in $(seq 0 20); do s="$s${s:+,}$i:$1"; done; echo "$s"; }
timeout -k 10 300 python tools/tune.py --dtype $DT --batch 1 --reps 7 --cands "" \
    "||UNET_MI355X_KSPLIT_FORCE=$(force 1)" "||UNET_MI355X_KSPLIT_FORCE=$(force 2)" \
    "||UNET_MI355X_KSPLIT_FORCE=$(force 4)" "||UNET_MI355X_KSPLIT_FORCE=$(force 8)" \
    "||UNET_MI355X_KSPLIT_FORCE=$(force 16)" > gpurun_out/bs1_sweep_${TAG}_$DT.txt 2>&1
echo sweep ok
