#!/bin/bash
# pass-1 batching: numeric GPU tests + C5/C3 A/B of SDP_PASS1_BATCH; then the contiguous-L1 timing experiment
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edges.py tests/test_gpu_gk.py tests/test_gpu_multirank.py tests/test_gpu_ragged.py tests/test_gpu_sorted.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/r03aa_tests.log 2>&1 || { tail -30 gpurun_out/r03aa_tests.log; exit 1; }
tail -2 gpurun_out/r03aa_tests.log
for v in 0 1; do
  SDP_PASS1_BATCH=$v timeout -k 10 400 python -u tools/c5_profile.py > gpurun_out/r03aa_c5_b$v.log 2>&1 || { tail -20 gpurun_out/r03aa_c5_b$v.log; exit 1; }
  echo "c5 pass1_batch=$v"; grep -E "steps|sdp_pass1" gpurun_out/r03aa_c5_b$v.log | head -3
done
for v in 0 1; do
  SDP_PASS1_BATCH=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-plots > gpurun_out/r03aa_c3_b$v.json 2> gpurun_out/r03aa_c3_b$v.err || { tail -20 gpurun_out/r03aa_c3_b$v.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03aa_c3_b$v.json').read().strip().splitlines()[-1]);k=d['per_kernel'];print('c3 pass1_batch=$v', d['ms_per_step'], {x: round(k[x]['ms_per_step'],3) for x in k if 'pass1' in x})"
done
bash tools/gpu_lib_kb.sh l1c l1contig group f64_norm f32_uniform
