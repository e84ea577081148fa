#!/bin/bash
# Gram parity tests + C5 bench (no plots) -- logs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-c5}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_configs.py::test_c5_wide_pearson_2e5 \
    tests/test_gpu_parity.py::test_corr_reject -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 --no-plots > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err
rc=$?
tail -3 gpurun_out/${tag}_t.log
exit $rc
