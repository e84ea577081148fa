#!/bin/bash
# dedup v2: grouping tests + A/B (SDP_DEDUP_V2) of the grouping stage on 1e9-row columns
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03m}
timeout -k 10 300 python -u -m pytest tests/test_gpu_grouping.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1 || { tail -30 gpurun_out/${TAG}_t.log; exit 1; }
tail -2 gpurun_out/${TAG}_t.log
bash tools/gpu_env_abn.sh ${TAG} group SDP_DEDUP_V2 "0 1 2" f64_norm i64_zipf f32_uniform i64_uniform_2p31
