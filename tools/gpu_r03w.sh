#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
BENCH_ARGS="--rows 125000000 --no-plots" timeout -k 10 400 bash tools/gpu_gaps.sh r03w_one || exit 1
BENCH_ARGS="--rows 125000000" timeout -k 10 400 bash tools/gpu_gaps.sh r03w_oneplots
