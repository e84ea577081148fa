#!/bin/bash
# Byte-key grouping: parity tests, then per-column stage timings at 1e9 rows.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-bytes}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_grouping.py tests/test_gpu_ragged.py tests/test_gpu_parity.py::test_categorical \
    tests/test_gpu_configs.py::test_c4_high_cardinality_4m tests/test_gpu_configs.py::test_c3_bench_table_4m \
    > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
for c in str_card100 str_card1e5 str_card1e8; do
  timeout -k 10 240 python -u tools/kbench.py group 1000000000 2 $c > gpurun_out/${T}_kb_$c.log 2>&1 || exit 1
done
tail -n 9 gpurun_out/${T}_kb_*.log
