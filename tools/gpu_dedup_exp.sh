#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in f64_norm i64_zipf f32_uniform; do for d in 0 1; do
  SDP_DEDUP_DIRECT=$d timeout -k 10 300 python -u tools/kbench.py group 1000000000 3 $c > gpurun_out/dd_${c}_$d.log 2>&1 || { tail -5 gpurun_out/dd_${c}_$d.log; exit 1; }
  echo "$c direct=$d $(grep -E 'dedup' gpurun_out/dd_${c}_$d.log)"
done; done
