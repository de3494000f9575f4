#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
bash tools/x3_ab.sh r6b
bash tools/gpu_check.sh r6b
