# A/B of two library builds on one box: the base build (libunet_mi355x_base.so, made from an older
# tree with `make OUT=../unet_mi355x/libunet_mi355x_base.so`) vs the in-tree one -- bitwise logits
# (tools/lib_ab.py) and per-launch times (tools/tune.py), interleaved A B A B.  Results under gpurun_out/.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
BASE=$GRAFT_REPO_ROOT/tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x_base.so
TAG=${1:-exp}
UNET_MI355X_LIB=$BASE timeout -k 10 200 python tools/lib_ab.py --save gpurun_out/${TAG}_a.npz > gpurun_out/${TAG}_ab.txt 2>&1
timeout -k 10 200 python tools/lib_ab.py --save gpurun_out/${TAG}_b.npz --compare gpurun_out/${TAG}_a.npz >> gpurun_out/${TAG}_ab.txt 2>&1
echo ab ok
for i in 1 2; do
  UNET_MI355X_LIB=$BASE timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 > gpurun_out/${TAG}_tune_base$i.txt 2>&1
  timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 ${EXTRA_CANDS} > gpurun_out/${TAG}_tune_new$i.txt 2>&1
  echo tune $i ok
done
