#!/bin/bash
# FETCH_SIZE calibration passes over tools/calib/fetch_calib (one rocprofv3 run per counter group).
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/calib; mkdir -p $OUT
timeout -k 10 60 ./tools/calib/fetch_calib > $OUT/plain.txt 2>&1
i=0
for grp in "FETCH_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" \
           "TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/pass$i -o run -- \
      ./tools/calib/fetch_calib > $OUT/pass$i.log 2>&1
  echo "calib pass $i ok"
done
