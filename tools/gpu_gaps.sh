#!/bin/bash
# Kernel trace of a 1-step bench; idle-gap summary of the timed step.
set -o pipefail
TAG=${1:-gaps}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
f=$(find gpurun_out/${TAG}_kt -name '*kernel_trace.csv' | head -1)
ms=$(python3 -c "import json; print(json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1])['ms_per_step'])")
python3 tools/gap_summary.py "$f" "$ms" | tee gpurun_out/${TAG}_gaps.txt
gzip -c "$f" > gpurun_out/${TAG}_kernel_trace.csv.gz; rm -rf gpurun_out/${TAG}_kt
