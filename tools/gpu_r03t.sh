#!/bin/bash
# byte wave dedup: grouping/categorical/config tests + C3 1e9 A/B of SDP_DEDUP_BYTES_V2 + C5 profile
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03t}
timeout -k 10 600 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_configs.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for v in 0 1 0 1; do
  SDP_DEDUP_BYTES_V2=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-plots > gpurun_out/${TAG}_b$v.json 2> gpurun_out/${TAG}_b$v.err || { tail -20 gpurun_out/${TAG}_b$v.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/${TAG}_b$v.json').read().strip().splitlines()[-1]);k=d['per_kernel']
print('bytes_v2=$v step', d['ms_per_step'], ' '.join('%s %.3f' % (x, k[x]['ms_per_step']) for x in k if 'bytes' in x))" | tee -a gpurun_out/${TAG}_ab.log
done

