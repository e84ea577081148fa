#!/bin/bash
# Fixed-overhead probe: bench at 1/8 and 1/4 of the C3 rows (the per-rank share
# at 8 and 4 GPUs), then a kernel-trace gap census at 1/8 without plots.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
TAG=${1:-small}
for r in 125000000 250000000; do
timeout -k 10 300 python -u bench.py --rows $r --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$r.json 2> gpurun_out/${TAG}_$r.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/${TAG}_$r.json'));print($r,d['ms_per_step'],d['value'])"
done
[ "${GAPS:-1}" = 1 ] || exit 0
BENCH_ARGS="--rows 125000000 --no-plots" bash tools/gpu_gaps.sh ${TAG}_gaps
