#!/bin/bash
# The 8-GPU per-rank share on one GPU: bench at ROWS (default 1.25e8) single vs
# forced-sharded (SDP_FORCE_SHARDED=1: every sharded branch over a one-rank RCCL
# group), with the readback census; NOPROF unset adds a kernel-trace gap census.
# usage: tools/gpu_rank_share.sh TAG [ROWS]
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-share}; ROWS=${2:-125000000}
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows $ROWS --steps 5 --warmup 2 --no-cpu-baseline \
      > gpurun_out/${TAG}_share_$mode.json 2> gpurun_out/${TAG}_share_$mode.err \
      || { tail -20 gpurun_out/${TAG}_share_$mode.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_share_$mode.json').read().strip().splitlines()[-1]);print('rows $ROWS forced_sharded=$mode', d['ms_per_step'], 'ms, readbacks', d['host_readbacks_per_step'])"
done
[ -n "$NOPROF" ] && exit 0
BENCH_ARGS="--rows $ROWS --no-plots" bash tools/gpu_gaps.sh ${TAG}_gaps
