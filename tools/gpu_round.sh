set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_14.log 2>&1
timeout -k 10 300 python tools/tune.py --dtype bf16 --batch 256 --reps 3 --cands "" "|0:4,1:4,2:4,3:4" "|0:21,1:21,2:21,3:21" "|0:22,1:22,2:22,3:22" "|0:15,1:15,2:15,3:15" > gpurun_out/tune_14.txt 2>&1
UNET_MI355X_LIB=$GRAFT_REPO_ROOT/tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x_abl.so timeout -k 10 200 python tools/tune.py --dtype bf16 --batch 256 --reps 1 --cands "2:30,15:30,16:31" > gpurun_out/tune_stamp3.txt 2>&1
