#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SDP_PASS2_BATCH=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r03ae_tests.log 2>&1 || { tail -30 gpurun_out/r03ae_tests.log; exit 1; }
tail -2 gpurun_out/r03ae_tests.log
SDP_PASS2_BATCH=1 timeout -k 10 400 python -u tools/c5_profile.py > gpurun_out/r03ae_c5.log 2>&1 || { tail -20 gpurun_out/r03ae_c5.log; exit 1; }
head -12 gpurun_out/r03ae_c5.log
for v in 0 1; do
  SDP_PASS2_BATCH=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-plots > gpurun_out/r03ae_c3_b$v.json 2> gpurun_out/r03ae_c3_b$v.err || { tail -20 gpurun_out/r03ae_c3_b$v.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03ae_c3_b$v.json').read().strip().splitlines()[-1]);k=d['per_kernel'];print('c3 pass2_batch=$v', d['ms_per_step'], {x: round(k[x]['ms_per_step'],3) for x in k if 'pass2' in x})"
done
