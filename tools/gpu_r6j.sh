#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R128="0:2,1:2,2:2,3:2,4:2,5:2,6:2,7:2,8:2,9:2,10:2,11:2,12:2,13:2,14:2,15:2,16:2"
UNET_MI355X_CFG=$R128 timeout -k 10 400 python -u -m pytest tests/test_forward_gpu.py -x -v --timeout 120 \
    --timeout-method thread -k "(golden_logits or reference_512_logits or golden_intermediates or small_batch_split or bs32_fp32 or masks_512) and not exact" \
    > gpurun_out/gpu_tests_r6j.log 2>&1
echo "tests rc=$?"
grep -E "passed|failed" gpurun_out/gpu_tests_r6j.log | tail -1
timeout -k 10 300 python tools/tune.py --dtype fp32 --batch 32 --reps 3 --cands "" "$R128|" > gpurun_out/x3_tune_r6j.txt 2>&1
timeout -k 10 300 python tools/tune.py --dtype fp32 --batch 1 --reps 5 --cands "" "$R128|" > gpurun_out/x3_tune_bs1_r6j.txt 2>&1
echo tune ok
