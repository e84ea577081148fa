#!/bin/bash
# The whole GPU suite (no -x: every failure in one call) + smoke; logs under gpurun_out/.
# Usage (via gpurun): bash tools/gpu_full.sh TAG
set -o pipefail
TAG=${1:-full}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1050 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=15 \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
tail -40 gpurun_out/${TAG}_tests.log
cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_smoke.log; exit $rc
