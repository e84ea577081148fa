#!/bin/bash
# Per-rank fixed cost at the 8-GPU share: bench at 1.25e8 rows, the sync census
# (host<->device copies per step by call site) and a kernel-trace busy summary.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fc}
timeout -k 10 300 python -u bench.py --rows 125000000 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err &&
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('1.25e8', d['ms_per_step'])" &&
timeout -k 10 300 python -u tools/sync_census.py 125000000 > gpurun_out/${TAG}_census.txt 2>&1 &&
timeout -k 10 400 bash tools/gpu_prof_rows.sh ${TAG}p 125000000
