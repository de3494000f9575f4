#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/lib_ab.sh r6g fp32 32 '' nocarry ns3
timeout -k 10 200 python tools/tune.py --dtype fp32 --batch 1 --reps 5 --cands "" "||UNET_MI355X_F32X3=0" > gpurun_out/x3_tune_bs1_r6g.txt 2>&1
echo bs1 ok
