#!/bin/bash
# multi-rank tests (2 gloo ranks, 1 forced-sharded nccl rank) + 1.25e8-row bench single vs forced-sharded
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-shd}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -m gpu -v --timeout 500 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log
grep -E "MISMATCH|calls|MULTIRANK" gpurun_out/${TAG}_multirank.log | tail -12
[ $rc -eq 0 ] || exit $rc
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_125m_$mode.json 2> gpurun_out/${TAG}_125m_$mode.err || { tail -20 gpurun_out/${TAG}_125m_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_125m_$mode.json').read().strip().splitlines()[-1]);print('forced_sharded=$mode', d['ms_per_step'])"
done
