#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-sp}; ROWS=${2:-125000000}
timeout -k 10 300 python -u tools/step_profile.py $ROWS 1 > gpurun_out/${TAG}_sharded.txt 2>&1 || { tail -20 gpurun_out/${TAG}_sharded.txt; exit 1; }
head -3 gpurun_out/${TAG}_sharded.txt
timeout -k 10 300 python -u tools/step_profile.py $ROWS 0 > gpurun_out/${TAG}_single.txt 2>&1 || { tail -20 gpurun_out/${TAG}_single.txt; exit 1; }
head -3 gpurun_out/${TAG}_single.txt
