#!/bin/bash
# host profile of one 1.25e8-row step: single rank vs sharded paths forced over a one-rank nccl group
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03l}
for mode in 0 1; do
  timeout -k 10 300 python -u tools/step_profile.py 125000000 $mode 1 > gpurun_out/${TAG}_stepprof_$mode.log 2>&1 || { tail -20 gpurun_out/${TAG}_stepprof_$mode.log; exit 1; }
  grep "step ms" gpurun_out/${TAG}_stepprof_$mode.log
done
echo done
