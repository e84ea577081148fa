"""Per-column quantile-window plan of the C3 generator after numeric_pass1_batch
(sample sizes, exclusive mask, candidate share).  usage: python tools/dbg_windows_c3.py [rows]"""
import sys
sys.path.insert(0, 'spark-df-profiling_amd'); sys.path.insert(0, '.')
import torch
import bench
from spark_df_profiling.engine import Engine
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
t = bench.make_c3_shard(rows, 0, 1, torch.device('cuda'))
cols = [c for c in t.columns if c.kind == 'fixed' and c.spark_type != 'date']
e = Engine()
for c, (p1, plan, ci) in zip(cols, e.numeric_pass1_batch(cols)):
    n = max(1, p1['count'])
    cand = sum(p1['w_in'][w] for w in range(plan.n_windows))
    print('%-18s nw %d n_sample %7d excl %#x  candidates %.4f  w_in %s' % (
        c.name, plan.n_windows, plan.n_sample, plan.excl_mask, cand / n,
        [round(p1['w_in'][w] / n, 4) for w in range(plan.n_windows)]), flush=True)
