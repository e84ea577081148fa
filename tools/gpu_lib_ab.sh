#!/bin/bash
# bench.py with the default library vs build_ab/libsdp_$VARIANT.so (SDP_LIBRARY), alternating
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-lab}; V=${2}; KEYS=${3:-sdp_part_dedup[bytes]}
for lib in default $V default $V; do
  if [ $lib = default ]; then unset SDP_LIBRARY; else export SDP_LIBRARY=$PWD/build_ab/libsdp_$lib.so; fi
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-plots ${BENCH_ARGS} > gpurun_out/${TAG}_$lib.json 2> gpurun_out/${TAG}_$lib.err || { tail -20 gpurun_out/${TAG}_$lib.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$lib.json').read().strip().splitlines()[-1]);k=d['per_kernel']
print('$lib step', d['ms_per_step'], ' '.join('%s %.3f' % (x, k[x]['ms_per_step']) for x in '$KEYS'.split(',') if x in k))"
done
