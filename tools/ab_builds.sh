# A/B of library builds on one box: tools/lib_ab.py (bitwise logits of every build against the
# first) and tools/tune.py (per-launch times), the builds interleaved, two rounds.
#   bash tools/ab_builds.sh TAG [build ...]   build = suffix of libunet_mi355x_<build>.so, or "new" for
#                                            the in-tree libunet_mi355x.so (default: base new)
# Older trees are built with `make OUT=../unet_mi355x/libunet_mi355x_<build>.so`.  Results in gpurun_out/.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-exp}; shift || true
BUILDS=${*:-base new}
D=$GRAFT_REPO_ROOT/tw-invoice-unet-ocr-llm_amd/unet_mi355x
lib() { if [ "$1" = new ]; then echo $D/libunet_mi355x.so; else echo $D/libunet_mi355x_$1.so; fi; }
first=""
for b in $BUILDS; do
  if [ -z "$first" ]; then
    first=$b
    UNET_MI355X_LIB=$(lib $b) timeout -k 10 200 python tools/lib_ab.py --save gpurun_out/${TAG}_$b.npz > gpurun_out/${TAG}_ab_$b.txt 2>&1
  else
    UNET_MI355X_LIB=$(lib $b) timeout -k 10 200 python tools/lib_ab.py --save gpurun_out/${TAG}_$b.npz --compare gpurun_out/${TAG}_$first.npz > gpurun_out/${TAG}_ab_$b.txt 2>&1 || echo "ab $b: not bitwise (see ${TAG}_ab_$b.txt)"
  fi
  echo "ab $b ok"
done
rm -f gpurun_out/${TAG}_*.npz   # only the bitwise comparison reads them (and 4 builds' logits exceed gpurun's 64 MiB pull)
for i in 1 2; do
  for b in $BUILDS; do
    UNET_MI355X_LIB=$(lib $b) timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 > gpurun_out/${TAG}_tune_$b$i.txt 2>&1
    echo "tune $b $i ok"
  done
done
