#!/bin/bash
# BASELINE-size parity tests (C2 1e8, C4 1e9, C5 1e7, C3 1e9) on the box.
# Usage (via gpurun): bash tools/gpu_sizes.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-sizes}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${2:-}
timeout -k 10 1000 python -u -m pytest tests/test_gpu_baseline_sizes.py tests/test_gpu_scale_1e9.py -m gpu -x -v \
    --timeout 600 --timeout-method thread --durations=0 ${K:+-k "$K"} > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -30 gpurun_out/${TAG}_tests.log; exit $rc
