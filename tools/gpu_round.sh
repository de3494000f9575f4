#!/bin/bash
# One GPU-box pass: gpu tests + smoke, the default bench line, rocprofv3 kernel stats, PMC passes
# (HBM bytes: FETCH_SIZE / WRITE_SIZE; SQ: MFMA busy, LDS bank conflicts, waits), each in a run of
# its own (--pmc only with --kernel-trace).
# Usage (from this container, after committing):
#   gpurun --timeout 1200 -- "bash tools/gpu_round.sh TAG $(git rev-parse --short HEAD) [skip-tests]"
set -e
TAG=${1:-r3}
COMMIT=${2:-unknown}
MODE=${3:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$MODE" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo smoke ok
fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
timeout -k 10 300 python bench.py --size 1024 --batch 64 --dtype fp16 --steps 5 --warmup 3 --cpu-seconds 10 --no-latency \
    --no-strong > gpurun_out/bench_${TAG}_cfg5_fp16_1024.json 2> gpurun_out/bench_${TAG}_cfg5.err
echo bench cfg5 ok
P="--no-cpu-baseline --no-latency --no-strong --no-fp32"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 3 --warmup 1 $P > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err
echo prof ok
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-layer-profile $P > gpurun_out/pmc_$TAG/pass$i.log 2>&1
done
echo pmc ok
python tools/pmc_summary.py gpurun_out/pmc_$TAG --bench-json gpurun_out/prof_bench_$TAG.json --commit $COMMIT \
    --out gpurun_out/pmc_$TAG/summary.json > gpurun_out/pmc_$TAG/summary.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --min-grid 10000 > gpurun_out/prof_$TAG/summary.txt
echo summaries ok
# BASELINE config 5 (1024^2, fp16, bs64): kernel stats + the same PMC passes
C5="--size 1024 --batch 64 --dtype fp16 $P"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_cfg5 -o run -- \
    python3 bench.py --steps 3 --warmup 1 $C5 > gpurun_out/prof_bench_${TAG}_cfg5.json 2> gpurun_out/prof_${TAG}_cfg5.err
mkdir -p gpurun_out/pmc_${TAG}_cfg5
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_${TAG}_cfg5/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-layer-profile $C5 > gpurun_out/pmc_${TAG}_cfg5/pass$i.log 2>&1
done
python tools/pmc_summary.py gpurun_out/pmc_${TAG}_cfg5 --batch 64 --size 1024 --bench-json gpurun_out/prof_bench_${TAG}_cfg5.json \
    --commit $COMMIT --out gpurun_out/pmc_${TAG}_cfg5/summary.json > gpurun_out/pmc_${TAG}_cfg5/summary.txt
python tools/prof_summary.py gpurun_out/prof_${TAG}_cfg5/run_kernel_trace.csv --min-grid 10000 > gpurun_out/prof_${TAG}_cfg5/summary.txt
echo cfg5 profiles ok
