#!/bin/bash
# Round-4 probes, second set: batch-1 kernel configurations (the 4-wave 16x16-tile rings on the level-0/1
# layers: 2x the pixel tiles of the 8-wave ring), static wave priority at the bench shape, and the
# saddr-form weight DMA build against the current one (tools/ab_builds.sh).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r4}
timeout -k 10 200 python tools/tune.py --dtype mixed --batch 1 --reps 30 --cands "" "1:3,2:3,13:3,14:3" "1:3,2:3,13:3,14:3,15:4,16:4" "||UNET_MI355X_KSPLIT=0" > gpurun_out/${TAG}_bs1_cfgs_mixed.txt 2>&1
echo "bs1 cfgs ok"
timeout -k 10 300 python tools/tune.py --dtype mixed --batch 256 --reps 3 --cands "" "||UNET_MI355X_PRIO=1" > gpurun_out/${TAG}_prio.txt 2>&1
echo "prio ok"
UNET_MI355X_KSPLIT=0 bash tools/ab_builds.sh ${TAG}ab new sv r3
echo "probe2 ok"
# batch-1 drop-in latency breakdown (host vs device stages)
for dt in mixed fp32; do
  timeout -k 10 200 python tools/latency_breakdown.py --dtype $dt --reps 50 > gpurun_out/${TAG}_latency_$dt.json 2>&1
done
echo "latency ok"
# XCD-owned row tiles on bottleneck.3: HBM-side reads with and without (FETCH_SIZE per dispatch)
P="--steps 1 --warmup 0 --no-layer-profile --no-cpu-baseline --no-latency --no-strong --no-fp32 --no-cfg5"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_xcd_off -o run -- python3 bench.py $P > gpurun_out/${TAG}_xcd_off.log 2>&1
UNET_MI355X_XCDROWS=8 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_xcd_on -o run -- python3 bench.py $P > gpurun_out/${TAG}_xcd_on.log 2>&1
echo "xcd pmc ok"
