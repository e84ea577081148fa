#!/bin/bash
# Same-box A/B of whole C3 bench steps: bench.py (no CPU baseline) alternating
# between libraries, per-kernel HIP-event ms of the kernels that differ.
# usage: tools/gpu_bench_ab.sh TAG [REPS]   (LIBS="name=path ...", BENCH_ARGS)
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; REPS=${2:-2}
TREE=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so
LIBS=${LIBS:-"head=build_ab/libsdp_head.so tree=$TREE"}
for rep in $(seq $REPS); do
  for nl in $LIBS; do
    name=${nl%%=*}; L=${nl#*=}
    SDP_LIBRARY=$L timeout -k 10 400 python -u bench.py --no-cpu-baseline $BENCH_ARGS > gpurun_out/${T}_${name}_$rep.json \
        2> gpurun_out/${T}_${name}_$rep.err || { tail -5 gpurun_out/${T}_${name}_$rep.err; exit 1; }
    python3 - gpurun_out/${T}_${name}_$rep.json $name $rep >> gpurun_out/${T}_bench_ab.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pk = d['per_kernel']
print('%-5s rep %s  step %.2f ms  ' % (sys.argv[2], sys.argv[3], d['ms_per_step']) +
      '  '.join('%s %.2f' % (k, v['ms_per_step']) for k, v in sorted(pk.items()) if v['ms_per_step'] > 1.0))
PY
  done
done
cat gpurun_out/${T}_bench_ab.log
