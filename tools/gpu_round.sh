#!/bin/bash
# One GPU-box pass: gpu tests, default bench line, rocprofv3 kernel stats, PMC passes
# (HBM bytes: FETCH_SIZE / WRITE_SIZE; SQ: MFMA busy, LDS bank conflicts, waits), each in a run
# of its own (--pmc only with --kernel-trace).
# Usage (from this container): gpurun --timeout 1200 -- 'bash tools/gpu_round.sh TAG [skip-tests]'
set -e
TAG=${1:-r2}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo smoke ok
fi
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
timeout -k 10 300 python bench.py --size 1024 --batch 64 --dtype fp16 --steps 5 --warmup 3 --cpu-seconds 10 --no-latency \
    > gpurun_out/bench_${TAG}_cfg5_fp16_1024.json 2> gpurun_out/bench_${TAG}_cfg5.err
echo bench cfg5 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err
echo prof ok
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-layer-profile --no-latency > gpurun_out/pmc_$TAG/pass$i.log 2>&1
done
echo pmc ok
python tools/pmc_summary.py gpurun_out/pmc_$TAG --bench-json gpurun_out/prof_bench_$TAG.json --out gpurun_out/pmc_$TAG/summary.json > gpurun_out/pmc_$TAG/summary.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --min-grid 10000 > gpurun_out/prof_$TAG/summary.txt
echo summaries ok
