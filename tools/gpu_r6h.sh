#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_check.sh r6h
bash tools/bs1_sweep.sh r6h fp32
bash tools/lib_ab.sh r6h fp32 32 '' nohalo nosplit
