#!/bin/bash
# round-5 check: GPU suite, the row-scatter allocation probe, the 8-GPU rank
# share (single / forced-sharded) with the sync census by call site.
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05h}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/scatter_alloc_probe.py > gpurun_out/${TAG}_probe.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${TAG}_probe.log
export SDP_READBACK_SITES=1
NOPROF=1 bash tools/gpu_rank_share.sh ${TAG} || exit 1
grep "sync site" gpurun_out/${TAG}_share_1.err | head -40
