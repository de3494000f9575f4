#!/bin/bash
# One call: GPU tests on the in-tree build; then (pytest ended normally) a same-box A/B of the builds named
# (tools/ab_builds.sh) and the full measurement pass of tools/gpu_round.sh without its tests.
#   gpurun --timeout 1200 -- "bash tools/final_round.sh TAG COMMIT [build ...]"
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r3}; COMMIT=${2:-unknown}; shift 2 || true
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?
echo "tests rc $rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit $?
echo smoke ok
if [ $# -gt 0 ]; then bash tools/ab_builds.sh $TAG "$@" || exit $?; fi
bash tools/gpu_round.sh $TAG $COMMIT skip-tests
