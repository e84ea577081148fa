"""Host-side profile of one describe() step on the C3 table (cProfile, top entries).

    python tools/host_profile.py [rows] [plots:0|1]
    (SDP_FORCE_SHARDED=1: the sharded code paths over a one-rank RCCL group, as bench.py)
"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
import torch  # noqa: E402
from spark_df_profiling import plot  # noqa: E402
plot.start_pool()

import bench  # noqa: E402
from spark_df_profiling import describe  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10 ** 9
plots = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
dev = torch.device('cuda', 0)
torch.cuda.set_device(0)
comm = None
if os.environ.get('SDP_FORCE_SHARDED') == '1':
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    os.environ.setdefault('MASTER_PORT', '29611')
    os.environ.setdefault('RANK', '0')
    os.environ.setdefault('WORLD_SIZE', '1')
    dist.init_process_group('nccl', device_id=dev)
    from spark_df_profiling.comm import TorchComm
    comm = TorchComm()
t = bench.make_c3_shard(rows, 0, 1, dev)
describe(t, plots=plots, comm=comm)
torch.cuda.synchronize()
for p in (False, True):
    t0 = time.perf_counter()
    describe(t, plots=p, comm=comm)
    torch.cuda.synchronize()
    print('plots=%s step %.1f ms' % (p, (time.perf_counter() - t0) * 1e3), flush=True)
pr = cProfile.Profile()
pr.enable()
describe(t, plots=plots, comm=comm)
torch.cuda.synchronize()
pr.disable()
os.makedirs('gpurun_out', exist_ok=True)
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(70)
st.sort_stats('tottime').print_stats(30)
