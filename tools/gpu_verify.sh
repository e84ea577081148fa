#!/bin/bash
# GPU test suite, smoke and a short C3 bench; logs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-verify}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x \
    > gpurun_out/${T}_pytest_gpu.log 2>&1 &&
tail -5 gpurun_out/${T}_pytest_gpu.log &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 &&
echo "smoke ok" &&
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 > gpurun_out/${T}_c3_bench.json 2> gpurun_out/${T}_c3_bench.err &&
cat gpurun_out/${T}_c3_bench.json
