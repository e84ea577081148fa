"""Single-kernel driver for profiling: runs one engine stage on a 1e9-row column."""
import sys, os, time
sys.path.insert(0, 'spark-df-profiling_amd'); sys.path.insert(0, '.')
import torch, ctypes
import bench
from spark_df_profiling.engine import Engine
from spark_df_profiling import _native as nat
from spark_df_profiling._native import sdp, ptr

what = sys.argv[1]
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dev = torch.device('cuda')
t = bench.make_c3_shard(rows, 0, 1, dev)
cols = {c.name: c for c in t.columns}
e = Engine()
col = cols[sys.argv[4]] if len(sys.argv) > 4 else cols['f64_norm']
torch.cuda.synchronize()
for r in range(reps):
    rec = nat.start_recording() if r == reps - 1 else None
    t0 = time.perf_counter()
    if what == 'group':
        e.group(col, col.kind == 'bytes', dense=False)
    elif what == 'groupd':                   # the near-unique (direct) dedup mode describe() picks from its sample
        e._near_unique.add(id(col))
        e.group(col, False, dense=False)
    elif what == 'table':
        cap = int(os.environ['KB_CAP']) if os.environ.get('KB_CAP') else None
        e._distinct_fixed_table(col) if col.kind != 'bytes' else e.value_counts_bytes_table(col, capacity=cap)
    elif what == 'pass1':
        e.numeric_pass1(col)
    elif what == 'pass1b':                   # the describe() path: batched plans with refined windows
        e.numeric_pass1_batch([col])
    elif what == 'pass2':
        e.numeric_stats(col)
    elif what == 'p2count':                  # the describe() path: pass 1, then pass 2 + level-1 count
        packs = e.numeric_pass1_batch([col])
        e.numeric_stats_batch([col], packs, 10, [2], group_cols={0})
    elif what == 'p2countb':                 # the same for every column of the column's dtype (batched launch)
        same = [c for c in t.columns if c.kind == 'fixed' and c.dtype == col.dtype and c.spark_type != 'date']
        packs = e.numeric_pass1_batch(same)
        e.numeric_stats_batch(same, packs, 10, [2] * len(same), group_cols=set(range(len(same))))
    elif what == 'd32':                      # sdp_distinct32 (32-bit key spaces)
        lo = 0 if col.is_float else int(col.values[:rows].min().item())
        out = e._distinct32_launch(col, lo)
    elif what == 'sorted':                   # sdp_sorted_distinct (one streaming read), 5 launches
        out = torch.zeros(4, dtype=torch.int64, device=dev)
        cs = col.sdp()
        for _ in range(5):
            nat.annotate('sdp_sorted_distinct[%s]' % col.name, col.length * col.values.element_size())
            sdp.sdp_sorted_distinct(ctypes.byref(cs), ptr(out), nat.stream_handle())
    elif what == 'gram':
        num = [c for c in t.columns if c.kind == 'fixed' and c.spark_type != 'date']
        e.gram(num, [0.0] * len(num), [False] * len(num))
    torch.cuda.synchronize()
    print(what, col.name, 'rep', r, '%.2f ms' % ((time.perf_counter() - t0) * 1e3), flush=True)
    if rec is not None:
        nat.stop_recording()
        for k, v in rec.items():
            print('   %-40s %8.3f ms x%d' % (k, sum(a.elapsed_time(b) for a, b, _ in v), len(v)))
