"""Microbenchmark: global hash table vs radix-partitioned grouping per column."""
import sys, os, time, json
sys.path.insert(0, 'spark-df-profiling_amd'); sys.path.insert(0, '.')
import torch
import bench
from spark_df_profiling.engine import Engine

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
dev = torch.device('cuda')
t = bench.make_c3_shard(rows, 0, 1, dev)
e = Engine()
out = {}
for c in t.columns:
    res = {}
    for name, fn in (('table', lambda: (e.value_counts_bytes_table(c) if c.kind == 'bytes' else e._distinct_fixed_table(c))),
                     ('group', lambda: e.group(c, c.kind == 'bytes', dense=(c.kind == 'bytes')))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tab = fn()
        torch.cuda.synchronize()
        res[name] = (round((time.perf_counter() - t0) * 1e3, 2), None if tab is None else tab['groups'])
    out[c.name] = res
    print(c.name, res, flush=True)
