#!/bin/bash
# HBM traffic of the bench's sdp kernels from PMC counters (MI355X_MICROARCH.md
# "HBM [CDNA4]": FETCH_SIZE and WRITE_SIZE in separate passes, FETCH_SIZE x 2 on
# gfx950, both in KiB).  Counters only for kernels matching sdp:: (the
# generator's torch kernels are excluded).  Usage (via gpurun):
#   bash tools/gpu_traffic.sh TAG [ROWS]        (BENCH_ARGS: extra bench.py arguments, e.g. --workload c5)
# -> gpurun_out/TAG_traffic.json (copy to profiles/ to let bench.py report it)
set -o pipefail
TAG=${1:-traffic}
ROWS=${2:-1000000000}
cd "$(dirname "$0")/"..
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 420 rocprofv3 --kernel-trace --output-format csv --pmc $ctr --kernel-include-regex 'sdp::' \
      -d gpurun_out/pmc_$TAG/p$i -o run -- python3 bench.py --steps 1 --warmup 0 --rows $ROWS --no-cpu-baseline $BENCH_ARGS \
      > gpurun_out/pmc_$TAG/p$i.log 2>&1 || { echo "pass $ctr failed"; tail -5 gpurun_out/pmc_$TAG/p$i.log; exit 1; }
  echo "pmc pass $ctr ok"
done
WL=$(echo "$BENCH_ARGS" | sed -n "s/.*--workload[ =]\([a-z0-9]*\).*/\1/p")
python3 tools/traffic_summary.py gpurun_out/${TAG}_traffic.json $ROWS:${WL:-c3} gpurun_out/pmc_$TAG/p1 gpurun_out/pmc_$TAG/p2 || exit 1
rm -rf gpurun_out/pmc_$TAG
