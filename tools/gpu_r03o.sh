#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03o}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_grouping.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
SDP_FORCE_SHARDED=1 BENCH_ARGS="--rows 125000000 --no-plots" timeout -k 10 400 bash tools/gpu_gaps.sh ${TAG}_shd
