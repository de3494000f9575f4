#!/bin/bash
# A/B of library builds (make OUT=../unet_mi355x/libunet_mi355x_<name>.so BUILD=build_<name> EXTRA=...): the same
# tools/tune.py shape timed with each library in its own process, two rounds in alternation (same box).
# Usage: gpurun -- "bash tools/lib_ab.sh TAG DTYPE BATCH name1 name2 ..."   (name "" = the product library)
set -e
TAG=$1; DT=$2; B=$3; shift 3
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/lib_ab_$TAG.txt
: > $out
for r in 1 2; do
  for n in "$@"; do
    lib=tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x${n:+_$n}.so
    echo "== round $r lib ${n:-product}" >> $out
    UNET_MI355X_LIB=$PWD/$lib timeout -k 10 200 python tools/tune.py --dtype $DT --batch $B --reps 3 --cands "" \
        2>&1 | grep -E "TOTAL|conv4.0|down1.3|conv1.0" >> $out
  done
done
echo lib_ab ok
