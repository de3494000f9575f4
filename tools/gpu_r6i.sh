#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 --timeout-method thread \
    -k "retargets or eviction or survive or boundary_matches" > gpurun_out/gpu_tests_r6i.log 2>&1
echo "tests rc=$?"
bash tools/bs1_sweep.sh r6i fp32 && bash tools/lib_ab.sh r6i fp32 32 '' nohalo nosplit
