#!/bin/bash
# Timing-only ablation A/B on the GPU box: tools/tune.py on the ablation build (make -C
# tw-invoice-unet-ocr-llm_amd/csrc abl; never used for results), the candidates interleaved in one
# process, two rounds.  Candidates are tune.py's "<UNET_MI355X_CFG>|<UNET_MI355X_UPCFG>" strings; a
# ring configuration + 16 * k selects ablation k (csrc/unet_kernels.hip, conv3x3_ring8_kernel ABL).
#   gpurun -- "bash tools/abl_probe.sh TAG [--dtype mixed] -- CAND ..."
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; shift
ARGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ARGS+=("$1"); shift; done
shift || true
export UNET_MI355X_LIB=$GRAFT_REPO_ROOT/tw-invoice-unet-ocr-llm_amd/unet_mi355x/libunet_mi355x_abl.so
for i in 1 2; do
  timeout -k 10 300 python tools/tune.py --batch 256 --reps 3 "${ARGS[@]}" --cands "" "$@" > gpurun_out/${TAG}_abl$i.txt 2>&1
  echo "abl round $i ok"
done
