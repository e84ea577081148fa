#!/bin/bash
# Row-per-lane Gram (<= 12 columns): its tests, then kbench gram on the 1e9-row C3 table, rows vs MFMA tile.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r03ah}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_gram.py > gpurun_out/${T}_gram_tests.log 2>&1 || { tail -30 gpurun_out/${T}_gram_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gram_tests.log
for rep in 1 2; do
  for v in 1 0; do
    echo "== SDP_GRAM_ROWS=$v" >> gpurun_out/${T}_ab.log
    SDP_GRAM_ROWS=$v timeout -k 10 240 python -u tools/kbench.py gram 1000000000 3 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
  done
done
cat gpurun_out/${T}_ab.log
