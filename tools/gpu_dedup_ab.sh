#!/bin/bash
# dedup insert variants on the 1e9-row bench (production paths: DIRECT for near-unique columns)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-dab}
for v in 0 1 2 0; do
  SDP_DEDUP_MLP=$v timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-plots > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { tail -20 gpurun_out/${TAG}_$v.err; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/${TAG}_$v.json').read().strip().splitlines()[-1]);k=d['per_kernel']
print('mlp=$v step', d['ms_per_step'], 'dedup u64', k['sdp_part_dedup[u64]']['ms_per_step'], 'launches', k['sdp_part_dedup[u64]']['launches_per_step'])"
done
