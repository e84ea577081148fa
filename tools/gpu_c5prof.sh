#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-c5p}
timeout -k 10 400 python -u tools/c5_profile.py > gpurun_out/${TAG}_c5prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_c5prof.log; exit 1; }
head -30 gpurun_out/${TAG}_c5prof.log
