#!/bin/bash
# GPU tests, then the default bench at 1/2/3 column workers (no CPU baseline).
set -o pipefail
TAG=${1:-wk}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for w in ${WORKERS:-1 2 3}; do
  timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --workers $w > gpurun_out/${TAG}_w$w.json 2> gpurun_out/${TAG}_w$w.err || { tail -20 gpurun_out/${TAG}_w$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_w$w.json')); print('workers', $w, d['ms_per_step'], 'ms/step', d['value']/1e9, 'G rows/s', d['roofline']['kernel'], d['roofline']['frac'])"
done
