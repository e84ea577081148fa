#!/bin/bash
# Multirank parity (gloo, 2 ranks on one GPU), GPU tests, then bench at 1/8 and full size.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-cb}
TESTS=1 bash tools/gpu_multirank.sh || exit 1
for r in 125000000 1000000000; do
timeout -k 10 400 python -u bench.py --rows $r --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_$r.json 2> gpurun_out/${TAG}_$r.err || { tail -5 gpurun_out/${TAG}_$r.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_$r.json'));print($r,d['ms_per_step'],d['value'])"
done
