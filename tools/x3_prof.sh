#!/bin/bash
# The three-term fp32 plan's kernels: per-layer A/B timing and PMC counters (one pass per counter group).
set -e
TAG=${1:-x3p}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
bash tools/x3_ab.sh $TAG
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/pass$i -o run -- \
      python3 bench.py --dtype fp32 --batch 32 --steps 1 --warmup 0 --no-cpu-baseline --no-latency --no-strong \
      --no-fp32 --no-cfg5 --no-layer-profile --detail-out "" > gpurun_out/pmc_$TAG/pass$i.log 2>&1
done
echo pmc ok
