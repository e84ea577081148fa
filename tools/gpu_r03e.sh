#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03e}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_configs.py -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -8 gpurun_out/${TAG}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log
grep -E "OK world|MISMATCH|calls|MULTIRANK" gpurun_out/${TAG}_multirank.log | tail -30
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_r03d.sh ${TAG}
