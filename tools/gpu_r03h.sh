#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03h}
timeout -k 10 300 python -u -m pytest tests/test_gpu_sorted.py tests/test_gpu_parity.py -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_125m_$mode.json 2> gpurun_out/${TAG}_125m_$mode.err || { tail -20 gpurun_out/${TAG}_125m_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_125m_$mode.json').read().strip().splitlines()[-1]);print('forced_sharded=$mode', d['ms_per_step'])"
done
COLS="f64_norm str_card1e8" WHAT=group bash tools/gpu_pmc_group.sh ${TAG}
