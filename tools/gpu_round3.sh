#!/bin/bash
# Whole GPU suite + smoke + default bench + rocprof kernel stats + 1.25e8 single vs forced-sharded benches.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-rnd}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=12 > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -20 gpurun_out/${TAG}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG}_multirank.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['whole_profile'])"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
f=$(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${TAG}_kernel_stats.csv; rm -rf gpurun_out/${TAG}_prof
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_125m_$mode.json 2> gpurun_out/${TAG}_125m_$mode.err || { tail -20 gpurun_out/${TAG}_125m_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/${TAG}_125m_$mode.json').read().strip().splitlines()[-1]);print('125m forced_sharded=$mode', d['ms_per_step'])"
done
echo done
