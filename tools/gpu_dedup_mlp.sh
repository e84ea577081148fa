#!/bin/bash
# A/B of the dedup insert (SDP_DEDUP_MLP=0: one probe in flight per lane) on 1e9-row columns.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
TAG=${1:-mlp}
for c in f64_norm i64_zipf f32_uniform i64_uniform_2p31; do for d in 0 1; do
  SDP_DEDUP_MLP=$d timeout -k 10 300 python -u tools/kbench.py group 1000000000 3 $c > gpurun_out/${TAG}_${c}_$d.log 2>&1 || { tail -5 gpurun_out/${TAG}_${c}_$d.log; exit 1; }
  echo "$c mlp=$d $(grep -E 'dedup|rep 2' gpurun_out/${TAG}_${c}_$d.log | tr '\n' ' ')"
done; done
