#!/bin/bash
# GPU suite then the default bench (+ readback census) on the box; logs under gpurun_out/TAG_*.
# usage: tools/gpu_tb.sh TAG [pytest -k expr]
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-tb}
K=${2:+-k "$2"}
eval timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $K \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
NOPROF=1 bash tools/gpu_bench.sh $TAG
