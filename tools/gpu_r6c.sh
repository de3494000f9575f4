#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/x3_ab.sh r6c
bash tools/gpu_check.sh r6c
