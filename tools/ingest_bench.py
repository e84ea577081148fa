"""End-to-end (PCIe-inclusive) rates of the Arrow/Parquet staging pipeline on
the C3 column mix:

    python tools/ingest_bench.py [rows] [workdir]

  arrow_h2d     host Arrow table (already decoded) -> HBM: staging + PCIe only
  parquet_h2d   parquet file -> HBM: decode threads + staging + PCIe
  describe_e2e  describe('<file>.parquet'): ingest plus the whole profile

Prints one JSON line.  The synthetic table is the bench generator's, moved to
the host; the parquet file is written with 1 M-row row groups."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'spark-df-profiling_amd'))
sys.path.insert(0, ROOT)
import pyarrow.parquet as pq  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from spark_df_profiling import describe  # noqa: E402
from spark_df_profiling.ingest import from_arrow_streamed, from_parquet  # noqa: E402

rows = int(float(sys.argv[1])) if len(sys.argv) > 1 else 50_000_000
work = sys.argv[2] if len(sys.argv) > 2 else '/tmp'
dev = torch.device('cuda')
shard = bench.make_c3_shard(rows, 0, 1, dev)
table = bench.shard_to_arrow(shard)
del shard
torch.cuda.empty_cache()
host_bytes = table.nbytes
out = {'rows': rows, 'columns': table.num_columns, 'arrow_bytes': host_bytes}

for rep in range(2):                                   # first pass warms the allocator
    st = {}
    t = from_arrow_streamed(table, dev, stats=st)
    del t
out['arrow_h2d'] = {'rows_per_s': round(st['rows_per_s'], 1), 'gb_per_s': round(st['h2d_gbs'], 2),
                    'seconds': round(st['seconds'], 3)}

path = os.path.join(work, 'sdp_ingest_c3.parquet')
t0 = time.perf_counter()
pq.write_table(table, path, row_group_size=1 << 20)
out['parquet_write_s'] = round(time.perf_counter() - t0, 1)
out['parquet_bytes'] = os.path.getsize(path)
del table
for rep in range(2):
    st = {}
    t = from_parquet(path, device=dev, stats=st)
    del t
out['parquet_h2d'] = {'rows_per_s': round(st['rows_per_s'], 1), 'gb_per_s': round(st['h2d_gbs'], 2),
                      'seconds': round(st['seconds'], 3)}
torch.cuda.synchronize()
t0 = time.perf_counter()
describe(path, plots=False)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
out['describe_e2e'] = {'rows_per_s': round(rows / dt, 1), 'seconds': round(dt, 3)}
os.remove(path)
print(json.dumps(out), flush=True)
