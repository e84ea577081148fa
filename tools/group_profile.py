"""Per-column timing of the grouping stages (HIP events per entry point) on the
C3 table: python tools/group_profile.py [rows]"""
import sys
import time
sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
import torch  # noqa: E402
import bench  # noqa: E402
from spark_df_profiling import _native as nat  # noqa: E402
from spark_df_profiling.engine import Engine  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 9
t = bench.make_c3_shard(rows, 0, 1, torch.device('cuda'))
e = Engine()
import os
only = os.environ.get('COLS', '').split()
for col in t.columns:
    if col.spark_type == 'date' or col.name == 'i64_uniform_1e6' or (only and col.name not in only):
        continue
    isb = col.kind == 'bytes'
    e.group(col, isb, dense=isb)
    torch.cuda.synchronize()
    rec = nat.start_recording()
    t0 = time.perf_counter()
    tab = e.group(col, isb, dense=isb)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    nat.stop_recording()
    parts = ', '.join('%s=%.2f' % (k.replace('sdp_part_', ''), sum(a.elapsed_time(b) for a, b, _ in v))
                      for k, v in rec.items() if sum(a.elapsed_time(b) for a, b, _ in v) > 0.3)
    print('%-18s groups=%-11s wall=%7.2f ms | %s' % (col.name, tab['groups'] if tab else None, wall, parts), flush=True)
