#!/bin/bash
# One GPU-box pass: gpu tests + smoke, then per workload (the headline bs256 mixed, BASELINE config 5)
# rocprofv3 kernel stats, the PMC passes (HBM bytes: FETCH_SIZE / WRITE_SIZE; SQ: MFMA busy, LDS bank
# conflicts, waits; each pass a run of its own, --pmc only with --kernel-trace) and their summary,
# which is installed as the bench's roofline.traffic source (profiles/pmc_<dtype>_bs<B>[_<S>].json on
# the box) BEFORE the bench line runs, so the line's traffic comes from this commit.
# Usage (from this container, after committing):
#   gpurun --timeout 1200 -- "bash tools/gpu_round.sh TAG $(git rev-parse --short HEAD) [skip-tests|no-bench|bench-only]"
# (no-bench: tests, smoke and the profiles; bench-only: the two bench lines -- two calls within the time limit)
# Copy gpurun_out/pmc_TAG/summary.json -> profiles/pmc_mixed_bs256.json (_cfg5 ->
# profiles/pmc_fp16_bs64_1024.json, _fp32 -> profiles/pmc_fp32_bs32.json) afterwards.
set -e
TAG=${1:-r3}
COMMIT=${2:-unknown}
MODE=${3:-}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$MODE" != "skip-tests" ] && [ "$MODE" != "bench-only" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
  echo tests ok
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
  echo smoke ok
fi
P="--no-cpu-baseline --no-latency --no-strong --no-fp32 --no-cfg5"
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE")
profile() {   # profile SUFFIX TRAFFIC_JSON BENCH_ARGS...
  local S=$1 TJ=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG$S -o run -- \
      python3 bench.py --steps 3 --warmup 1 $P --detail-out gpurun_out/prof_bench_$TAG$S.detail.json "$@" \
      > gpurun_out/prof_bench_$TAG$S.json 2> gpurun_out/prof_$TAG$S.err
  mkdir -p gpurun_out/pmc_$TAG$S
  local i=0
  for grp in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG$S/pass$i -o run -- \
        python3 bench.py --steps 1 --warmup 0 --no-layer-profile $P --detail-out "" "$@" > gpurun_out/pmc_$TAG$S/pass$i.log 2>&1
  done
  python tools/pmc_summary.py gpurun_out/pmc_$TAG$S --bench-json gpurun_out/prof_bench_$TAG$S.detail.json --commit $COMMIT \
      --out gpurun_out/pmc_$TAG$S/summary.json "${SUMARGS[@]}" > gpurun_out/pmc_$TAG$S/summary.txt
  python tools/prof_summary.py gpurun_out/prof_$TAG$S/run_kernel_trace.csv --min-grid 10000 > gpurun_out/prof_$TAG$S/summary.txt
  cp gpurun_out/pmc_$TAG$S/summary.json "profiles/$TJ"
}
if [ "$MODE" != "bench-only" ]; then
SUMARGS=()
profile "" pmc_mixed_bs256.json
echo profiles ok
# every traffic source of the bench line (headline, config 5, fp32 leg) from this commit before it runs
SUMARGS=(--batch 64 --size 1024)
profile _cfg5 pmc_fp16_bs64_1024.json --size 1024 --batch 64 --dtype fp16
echo cfg5 profiles ok
SUMARGS=(--batch 32 --esize 4)
profile _fp32 pmc_fp32_bs32.json --batch 32 --dtype fp32
echo fp32 profiles ok
fi
[ "$MODE" = "no-bench" ] && exit 0
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --detail-out gpurun_out/bench_$TAG.detail.json \
    > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
# the profiles of this pass against the bench line of the same box (tools/stamp_profiles.py)
if [ "$MODE" != "bench-only" ]; then
  python tools/stamp_profiles.py --tag $TAG --commit $COMMIT --stats gpurun_out/prof_$TAG/run_kernel_stats.csv \
      --pmc gpurun_out/pmc_$TAG/summary.json --bench gpurun_out/bench_$TAG.json --out gpurun_out/stamp_$TAG.json \
      > /dev/null && echo stamp ok
fi
timeout -k 10 300 python bench.py --size 1024 --batch 64 --dtype fp16 --steps 5 --warmup 3 --cpu-seconds 10 --no-latency \
    --no-strong --detail-out gpurun_out/bench_${TAG}_cfg5.detail.json > gpurun_out/bench_${TAG}_cfg5_fp16_1024.json 2> gpurun_out/bench_${TAG}_cfg5.err
echo bench cfg5 ok
