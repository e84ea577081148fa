"""One C5 describe() step (1e7 x 512 fp32, no plots): wall time, the kernel
time per stage label (libsdp entry points, HIP events) and a cProfile of the
package's host functions.   python tools/c5_profile.py [rows] [cols]"""
import cProfile
import pstats
import sys
import time
from collections import defaultdict

sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
import torch  # noqa: E402

import bench  # noqa: E402
from spark_df_profiling import describe  # noqa: E402
from spark_df_profiling import _native as nat  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 7
ncols = int(sys.argv[2]) if len(sys.argv) > 2 else 512
dev = torch.device('cuda', 0)
t = bench.make_c5_shard(rows, 0, 1, dev, ncols=ncols)
describe(t, plots=False)
torch.cuda.synchronize()
walls = []
for _ in range(3):
    t0 = time.perf_counter()
    describe(t, plots=False)
    torch.cuda.synchronize()
    walls.append((time.perf_counter() - t0) * 1e3)
print('steps (ms):', ' '.join('%.1f' % w for w in walls))
rec = nat.start_recording()
t0 = time.perf_counter()
describe(t, plots=False)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) * 1e3
nat.stop_recording()
tot = defaultdict(lambda: [0.0, 0])
for k, v in rec.items():
    name = k.split('[')[0]
    tot[name][0] += sum(a.elapsed_time(b) for a, b, _ in v)
    tot[name][1] += len(v)
print('step %.1f ms, libsdp kernel time %.1f ms in %d calls' % (wall, sum(x[0] for x in tot.values()),
                                                                 sum(x[1] for x in tot.values())))
for name, (ms, c) in sorted(tot.items(), key=lambda kv: -kv[1][0])[:25]:
    print('  %-36s %8.2f ms  %6d calls' % (name, ms, c))
pr = cProfile.Profile()
pr.enable()
describe(t, plots=False)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(r'spark_df_profiling', 30)
st.sort_stats('tottime').print_stats(20)
