#!/bin/bash
# GPU tests, then kernel-trace stats of the grouping stages on 1e9-row C3 columns.
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for c in ${COLS:-f64_norm str_card1e8}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_$c -o run -- python3 tools/kbench.py group 1000000000 3 $c > gpurun_out/kt_$c.log 2>&1
  grep -E "rep" gpurun_out/kt_$c.log
  f=$(find gpurun_out/kt_$c -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/kstats_$c.csv
  rm -rf gpurun_out/kt_$c
done
