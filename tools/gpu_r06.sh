#!/bin/bash
# Round-6 GPU step: the grouping-related GPU tests, then same-box A/Bs of an
# environment switch on kbench stages and whole C3 bench steps.
# usage: tools/gpu_r06.sh TAG "SET_A SET_B" [TESTS] ; REPS, STEPS, COLS, STAGES
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; SETS=$2; TESTS=${3:-}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS \
      > gpurun_out/${T}_tests.log 2>&1; rc=$?
  tail -4 gpurun_out/${T}_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for st in ${STAGES:-}; do
  for c in ${COLS:-f64_norm}; do
    for v in $SETS; do
      echo "== $v $st $c" >> gpurun_out/${T}_kb.log
      env ${v//,/ } timeout -k 10 240 python -u tools/kbench.py $st 1000000000 2 $c 2>&1 \
          | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_kb.log || exit 1
    done
  done
done
[ -f gpurun_out/${T}_kb.log ] && cat gpurun_out/${T}_kb.log
for rep in $(seq ${REPS:-0}); do
  for v in $SETS; do
    env ${v//,/ } timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps ${STEPS:-5} --warmup 2 \
        > gpurun_out/${T}_${v//[=,]/_}_$rep.json 2> gpurun_out/${T}_${v//[=,]/_}_$rep.err \
        || { tail -5 gpurun_out/${T}_${v//[=,]/_}_$rep.err; exit 1; }
    python3 - gpurun_out/${T}_${v//[=,]/_}_$rep.json "$v" $rep >> gpurun_out/${T}_bench_ab.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = d['per_kernel']
print('%-16s rep %s  step %.2f ms  ' % (sys.argv[2], sys.argv[3], d['ms_per_step']) +
      '  '.join('%s %.2f' % (k, v['ms_per_step']) for k, v in sorted(pk.items()) if v['ms_per_step'] > 1.0))
PY
  done
done
[ -f gpurun_out/${T}_bench_ab.log ] && cat gpurun_out/${T}_bench_ab.log
exit 0
