"""Row-scatter time vs. where its 8-byte records land in HBM (verdict r04
item 4: the level-1 row scatter of a 1e9-row f64 column moves 26-42 ms per
C3 step between boxes and between runs on one box).  Runs the partitioning
countDistinct of one 1e9-row f64 column (bench.py's f64_norm) under several
allocator states and prints the level-1 row scatter's HIP-event time:

  warm        the caching allocator's blocks reused (the bench steady state)
  fresh       torch.cuda.empty_cache() first: new hipMalloc segments
  fragmented  after allocating and freeing an interleaved pattern of 2-3 GB blocks
  arena       records in one large buffer allocated once, offset 0 / 3 GB
                                                     (views, no allocator)

usage: python tools/scatter_alloc_probe.py [rows]"""
import os
import sys
import time

sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
import torch  # noqa: E402

import bench  # noqa: E402
from spark_df_profiling import _native as nat  # noqa: E402
from spark_df_profiling.engine import Engine  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
dev = torch.device('cuda')
t = bench.make_c3_shard(rows, 0, 1, dev)
keep = {'f64_norm'}
for c in list(t.columns):
    if c.name not in keep:
        c.values = c.validity = c.offsets = c.data = None
col = [c for c in t.columns if c.name == 'f64_norm'][0]
torch.cuda.empty_cache()
e = Engine()


def run(tag):
    rec = nat.start_recording()
    t0 = time.perf_counter()
    e.group(col, False, dense=False)
    torch.cuda.synchronize()
    nat.stop_recording()
    out = {k: sum(a.elapsed_time(b) for a, b, _ in v) for k, v in rec.items() if k.startswith('sdp_part')}
    sc = [v for k, v in out.items() if 'scatter' in k and 'rows' in k]
    print('%-22s total %.2f ms  rows-scatter %.3f ms  recs-scatter %.3f  dedup %.3f' % (
        tag, (time.perf_counter() - t0) * 1e3, sc[0] if sc else -1,
        sum(v for k, v in out.items() if k.startswith('sdp_part_recs') and 'scatter' in k),
        sum(v for k, v in out.items() if k.startswith('sdp_part_dedup'))), flush=True)


for i in range(3):
    run('warm %d' % i)
torch.cuda.empty_cache()
run('fresh')
run('fresh+warm')
# fragmentation: interleaved 2 / 3 GB blocks, every other one freed
blocks = [torch.empty((2 + i % 2) << 30, dtype=torch.uint8, device=dev) for i in range(24)]
for i in range(0, len(blocks), 2):
    blocks[i] = None
run('fragmented')
run('fragmented+warm')
blocks = None
torch.cuda.empty_cache()
# arena: the records in views of one big buffer
orig = e._records
arena = torch.empty(20 << 30, dtype=torch.uint8, device=dev)
for off in (0, 3 << 30):
    cur = [off]

    def records(nrec, isb, cur=cur):
        n8 = max(int(nrec), 1) * 8
        a = arena[cur[0]:cur[0] + n8].view(torch.int64)
        cur[0] += (n8 + (1 << 21) - 1) // (1 << 21) * (1 << 21)
        return nat.SdpRecords(a.data_ptr(), None, None), a
    e._records = records
    run('arena +%dG' % (off >> 30))
    cur[0] = off
    run('arena +%dG again' % (off >> 30))
e._records = orig
print('alloc conf', os.environ.get('PYTORCH_HIP_ALLOC_CONF'), flush=True)
