#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_r03m.sh r03n || exit 1
SDP_FORCE_SHARDED=1 BENCH_ARGS="--rows 125000000 --no-plots" timeout -k 10 400 bash tools/gpu_gaps.sh r03n_shd || exit 1
BENCH_ARGS="--rows 125000000 --no-plots" timeout -k 10 400 bash tools/gpu_gaps.sh r03n_one
