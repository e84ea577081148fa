#!/bin/bash
# Round validation on the box: the GPU suite, smoke(), the default bench with a
# rocprofv3 kernel-stats pass, and the 8-GPU rank share (1.25e8 rows) single vs
# forced-sharded.  -> gpurun_out/TAG_*
# usage: tools/gpu_round.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rnd}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=12 \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -20 gpurun_out/${TAG}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
bash tools/gpu_bench.sh $TAG || exit 1
NOPROF=1 bash tools/gpu_rank_share.sh $TAG || exit 1
