#!/bin/bash
# scratch GPU pass (edited per call)
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
bash tools/gpu_check.sh r6n
timeout -k 10 200 python tools/tune.py --dtype fp32 --batch 32 --reps 3 --cands "" > gpurun_out/x3s_tune_bs32_r6n.txt 2>&1
timeout -k 10 200 python tools/tune.py --dtype fp32 --batch 1 --reps 7 --cands "" > gpurun_out/x3s_tune_bs1_r6n.txt 2>&1
echo tune ok
