#!/bin/bash
# GPU tests, then (only if pytest ended normally: 0 = passed, 1 = test failures) the first-step probe,
# a driver-shaped bench line and the same-box A/B of two builds.  Stops at any other exit status
# (a fault, an abort, a time limit): nothing more runs on the GPU in that call.
#   gpurun --timeout 1200 -- "bash tools/check_then_ab.sh TAG [build ...]"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-exp}; shift || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -u tools/first_step_probe.py --trials 5 > gpurun_out/probe_$TAG.log 2>&1 || exit $?
echo probe ok
timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-latency --no-fp32 --no-strong \
    > gpurun_out/probe_bench_$TAG.json 2> gpurun_out/probe_bench_$TAG.err || exit $?
echo bench ok
bash tools/ab_builds.sh $TAG "$@"
