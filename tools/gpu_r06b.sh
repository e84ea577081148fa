#!/bin/bash
# Round-6 GPU step: the whole -m gpu suite, then a head/tree A/B of kbench
# stages (tools/gpu_ab.sh), then a short bench.py run.
# usage: tools/gpu_r06b.sh TAG "STAGE:COL ..." ; SKIP_TESTS=1, BENCH_STEPS (0: none)
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
      > gpurun_out/${T}_tests.log 2>&1; rc=$?
  tail -4 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for sc in $2; do
  LIBS=${LIBS:-"head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so"} \
    bash tools/gpu_ab.sh $T ${sc%%:*} ${sc#*:} > /dev/null || exit 1
done
[ -f gpurun_out/${T}_ab.log ] && grep -v "^ " gpurun_out/${T}_ab.log | grep -v "rep 0\b" | head -80
if [ "${BENCH_STEPS:-10}" != 0 ]; then
  timeout -k 10 400 python -u bench.py --steps ${BENCH_STEPS:-10} --warmup 2 > gpurun_out/${T}_bench.json \
      2> gpurun_out/${T}_bench.err || { tail -5 gpurun_out/${T}_bench.err; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('gpurun_out/${T}_bench.json').read().strip().splitlines()[-1])
print('step %.2f ms value %.3e frac %s' % (d['ms_per_step'], d['value'], d.get('roofline',{}).get('frac')))
for k,v in sorted(d['per_kernel'].items(), key=lambda kv:-kv[1]['ms_per_step'])[:25]: print('  %-45s %7.2f' % (k, v['ms_per_step']))"
fi
exit 0
