#!/bin/bash
# Pass-1 per-kernel times (kbench) on three column types, then the GPU round.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-p1}
for c in f64_norm f32_norm i64_zipf; do
timeout -k 10 120 python -u tools/kbench.py pass1 1000000000 3 $c > gpurun_out/${TAG}_kb_$c.log 2>&1 || { tail -20 gpurun_out/${TAG}_kb_$c.log; exit 1; }
tail -4 gpurun_out/${TAG}_kb_$c.log
done
bash tools/gpu_round.sh $TAG
