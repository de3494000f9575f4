#!/bin/bash
# rocprofv3 kernel stats + the three PMC passes of tools/gpu_round.sh for ONE bench configuration, and
# the PMC summary installed as that configuration's roofline.traffic source.
#   gpurun --timeout 900 -- "bash tools/pmc_config.sh TAG COMMIT OUT_JSON BATCH SIZE [bench args ...]"
#   e.g. ESIZE=4 bash tools/pmc_config.sh r3fp32 abc1234 pmc_fp32_bs32.json 32 512 --dtype fp32 --batch 32
# (ESIZE: bytes per stored element for the algorithmic-bytes column, default 2)
# (OUT_JSON: the name bench.py's kernel_table looks up, profiles/pmc_<dtype>_bs<B>[_<S>].json)
set -e
TAG=$1; COMMIT=$2; TJ=$3; BATCH=$4; SIZE=$5; shift 5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P="--no-cpu-baseline --no-latency --no-strong --no-fp32"
PASSES=("FETCH_SIZE" "WRITE_SIZE"
        "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE")
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- \
    python3 bench.py --steps 3 --warmup 1 $P "$@" > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_$TAG.err
echo prof ok
mkdir -p gpurun_out/pmc_$TAG
i=0
for grp in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d gpurun_out/pmc_$TAG/pass$i -o run -- \
      python3 bench.py --steps 1 --warmup 0 --no-layer-profile $P "$@" > gpurun_out/pmc_$TAG/pass$i.log 2>&1
  echo pass $i ok
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG --bench-json gpurun_out/prof_bench_$TAG.json --commit $COMMIT \
    --out gpurun_out/pmc_$TAG/summary.json --batch $BATCH --size $SIZE --esize ${ESIZE:-2} > gpurun_out/pmc_$TAG/summary.txt
python tools/prof_summary.py gpurun_out/prof_$TAG/run_kernel_trace.csv --min-grid 1000 > gpurun_out/prof_$TAG/summary.txt
cp gpurun_out/pmc_$TAG/summary.json "profiles/$TJ"
# the bench line of this configuration, now with its traffic
timeout -k 10 300 python bench.py --steps 10 --warmup 3 $P "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
echo bench ok
