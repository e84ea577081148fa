#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_ingest.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/r03x_tests.log 2>&1 || { tail -30 gpurun_out/r03x_tests.log; exit 1; }
tail -2 gpurun_out/r03x_tests.log
BENCH_ARGS="--rows 125000000 --no-plots" timeout -k 10 400 bash tools/gpu_gaps.sh r03x_one || exit 1
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03x_125m_$mode.json 2> gpurun_out/r03x_125m_$mode.err || { tail -20 gpurun_out/r03x_125m_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03x_125m_$mode.json').read().strip().splitlines()[-1]);print('125m forced_sharded=$mode', d['ms_per_step'])"
done
