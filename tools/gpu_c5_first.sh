#!/bin/bash
# First C5 look: fp64 MFMA peak, GPU tests, C5 bench at 1e6 then 1e7 rows.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ubench/mfma_f64_peak > gpurun_out/mfma_peak.json 2>&1 &&
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --workload c5 --rows 1000000 --steps 2 --warmup 1 > gpurun_out/c5_1e6.json 2> gpurun_out/c5_1e6.err &&
timeout -k 10 400 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/c5_1e7.json 2> gpurun_out/c5_1e7.err
echo "exit $?"
