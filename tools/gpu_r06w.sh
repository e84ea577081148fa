#!/bin/bash
# A/B of the sharded exchange's owner order at the 1.25e8-row rank share,
# forced-sharded: HEAD's torch sort/searchsorted/cumsum (build_ab/distributed_head.py
# + build_ab/comm_head.py in a copy of the tree) vs sdp_owner_order; bench timing + rocprofv3 kernel stats.
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=$PWD/gpurun_out
rm -rf /tmp/head_tree && mkdir /tmp/head_tree && cp -r bench.py __graft_entry__.py spark-df-profiling_amd oracle tests tools /tmp/head_tree/ \
  && cp build_ab/distributed_head.py /tmp/head_tree/spark-df-profiling_amd/spark_df_profiling/distributed.py \
  && cp build_ab/comm_head.py /tmp/head_tree/spark-df-profiling_amd/spark_df_profiling/comm.py || exit 1
for rep in ${REPS:-1 2}; do
for leg in head new; do
  d=$PWD; [ $leg = head ] && d=/tmp/head_tree
  (cd $d && SDP_FORCE_SHARDED=1 timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline \
      > $OUT/${TAG:-r06w}_${leg}_$rep.json 2> $OUT/${TAG:-r06w}_${leg}_$rep.err) || { tail -20 $OUT/${TAG:-r06w}_${leg}_$rep.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/${TAG:-r06w}_${leg}_$rep.json').read().strip().splitlines()[-1]);print('$leg rep $rep', d['ms_per_step'], 'ms')"
done
done
[ -n "$NOPROF" ] && exit 0
for leg in head new; do
  d=$PWD; [ $leg = head ] && d=/tmp/head_tree
  (cd $d && SDP_FORCE_SHARDED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/${TAG:-r06w}_prof_$leg -o run -- \
      python3 -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/${TAG:-r06w}_prof_$leg.log 2>&1) \
      || { tail -20 $OUT/${TAG:-r06w}_prof_$leg.log; exit 1; }
  f=$(find $OUT/${TAG:-r06w}_prof_$leg -name '*kernel_stats.csv' | head -1); cp "$f" $OUT/${TAG:-r06w}_${leg}_kernel_stats.csv
  rm -rf $OUT/${TAG:-r06w}_prof_$leg
done
echo done
