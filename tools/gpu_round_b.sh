#!/bin/bash
# GPU tests, then C5 and C3 benches -- logs under gpurun_out/<tag>_*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-b}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -x \
    > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -15 gpurun_out/${tag}_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workload c5 --steps 2 --warmup 1 > gpurun_out/${tag}_c5.json 2> gpurun_out/${tag}_c5.err &&
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${tag}_c3.json 2> gpurun_out/${tag}_c3.err
