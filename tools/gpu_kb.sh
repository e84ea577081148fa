#!/bin/bash
# Grouping tests + per-kernel times of one stage on chosen 1e9-row bench columns.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-kb}; STAGE=${2:-group}; shift 2
timeout -k 10 400 python -u -m pytest tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_configs.py \
    -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t.log 2>&1 || { tail -30 gpurun_out/${T}_t.log; exit 1; }
tail -2 gpurun_out/${T}_t.log
for c in "$@"; do
  timeout -k 10 200 python -u tools/kbench.py $STAGE 1000000000 3 $c > gpurun_out/${T}_$c.log 2>&1 || { tail -5 gpurun_out/${T}_$c.log; exit 1; }
  tail -8 gpurun_out/${T}_$c.log
done
