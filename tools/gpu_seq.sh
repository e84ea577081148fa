#!/bin/bash
# per-dispatch durations of chosen kernels over bench.py's steps (rocprofv3 kernel trace)
# usage: tools/gpu_seq.sh TAG PATTERN...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr -o run \
    -- python3 bench.py $BENCH_ARGS --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}.err \
    || { tail -20 gpurun_out/${TAG}.err; exit 1; }
f=$(find gpurun_out/${TAG}_tr -name '*kernel_trace.csv' | head -1)
python3 tools/dispatch_seq.py "$f" "$@" > gpurun_out/${TAG}_seq.txt
rm -rf gpurun_out/${TAG}_tr
cat gpurun_out/${TAG}_seq.txt | cut -c1-2000
