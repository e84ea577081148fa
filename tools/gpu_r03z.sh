#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_ragged.py tests/test_gpu_edges.py tests/test_gpu_sorted.py tests/test_gpu_gram.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/r03z_tests.log 2>&1 || { tail -30 gpurun_out/r03z_tests.log; exit 1; }
tail -2 gpurun_out/r03z_tests.log
bash tools/gpu_lib_ab.sh r03z oldmix "sdp_pass2_count[f64],sdp_pass2_count[f32],sdp_pass2_count[i64],sdp_part_rows[f64/scatter],sdp_part_rows[i64/scatter],sdp_part_rows[f32/scatter],sdp_part_recs[u64/scatter],sdp_part_dedup[u64],sdp_gram"
