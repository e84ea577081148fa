#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 16 7 12; do
  SDP_RECS_RPT=$r timeout -k 10 300 python -u tools/kbench.py group 1000000000 3 f64_norm > gpurun_out/recs_$r.log 2>&1 || { tail -5 gpurun_out/recs_$r.log; exit 1; }
  echo "rpt $r"; grep -E "rep 2|scatter|dedup|count" gpurun_out/recs_$r.log
done
for c in str_card1e8 str_card1e5; do
  for m in table group; do
    timeout -k 10 300 python -u tools/kbench.py $m 125000000 3 $c > gpurun_out/kb_${m}_$c.log 2>&1 || { tail -5 gpurun_out/kb_${m}_$c.log; exit 1; }
    echo "$m $c"; grep -E "rep 2" gpurun_out/kb_${m}_$c.log
  done
done
