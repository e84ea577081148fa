#!/bin/bash
# bench.py's default command (or BENCH_ARGS) plus a rocprofv3 kernel-stats pass of
# the same command, on the box.  -> gpurun_out/TAG_bench.json, TAG_kernel_stats.csv
# usage: tools/gpu_bench.sh TAG           (BENCH_ARGS="--workload c5" etc.; NOPROF=1 skips rocprof)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bench}
timeout -k 10 600 python -u bench.py $BENCH_ARGS > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
    || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python3 - "$TAG" <<'EOF'
import json, sys
d = json.loads(open('gpurun_out/%s_bench.json' % sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
print('bench', d['ms_per_step'], 'ms', d['value'], r['kernel'], r['frac'], r.get('whole_profile'),
      'readbacks', d.get('host_readbacks_per_step'))
EOF
[ -n "$NOPROF" ] && exit 0
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run \
    -- python3 bench.py $BENCH_ARGS --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err \
    || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv && rm -rf gpurun_out/${TAG}_prof
head -12 gpurun_out/${TAG}_kernel_stats.csv | cut -c1-160
