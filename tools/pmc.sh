#!/bin/bash
# PMC passes over one bench.py step (run ON the GPU box via gpurun, from the repo root).
# Each counter group gets its own rocprofv3 pass (--pmc only with --kernel-trace, never
# combined with sys/runtime traces).  Output: gpurun_out/pmc_<tag>/pass<i>/...
set -e
TAG=${1:-r1}
shift || true
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 400 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-layer-profile "$@" > $OUT/pass$i.log 2>&1
done
echo pmc done
