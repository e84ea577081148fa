#!/bin/bash
# Gram overlap: correctness (configs, parity, multirank) + C3 1e9 A/B of SDP_GRAM_OVERLAP
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03r}
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_gram.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for v in 0 1 0 1; do
  SDP_GRAM_OVERLAP=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_ov$v.json 2> gpurun_out/${TAG}_ov$v.err || { tail -20 gpurun_out/${TAG}_ov$v.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_ov$v.json').read().strip().splitlines()[-1]);print('overlap=$v', d['ms_per_step'], d['per_kernel']['sdp_gram']['ms_per_step'])" | tee -a gpurun_out/${TAG}_ab.log
done
