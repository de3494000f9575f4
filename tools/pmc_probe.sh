#!/bin/bash
# Extra PMC passes (one rocprofv3 run per counter group) over one bench step, for bottleneck
# probes beyond tools/gpu_round.sh's set.  Usage (on the GPU box via gpurun):
#   bash tools/pmc_probe.sh TAG "GROUP1 COUNTERS" "GROUP2 COUNTERS" ...
# Writes gpurun_out/pmcx_<TAG>/pass<i>/ and the available-counter list (once per tag).
set -e
TAG=$1; shift
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/pmcx_$TAG; mkdir -p $OUT
if [ ! -f $OUT/avail.txt ]; then
  timeout -s KILL 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || echo "list-avail failed"
fi
i=0
P="--no-cpu-baseline --no-latency --no-strong --no-fp32 --no-layer-profile"
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 $P > $OUT/pass$i.log 2>&1
  echo "pass $i ok: $grp"
done
