"""cProfile of one describe() step of the C3 table (optionally with the sharded
paths forced over a one-rank nccl group), restricted to the package's own
functions: where the host time of a step goes (kernel time shows up inside the
blocking readbacks).
    python tools/step_profile.py ROWS [sharded:0|1] [plots:0|1]"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, 'spark-df-profiling_amd')
sys.path.insert(0, '.')
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125_000_000
sharded = len(sys.argv) > 2 and sys.argv[2] == '1'
plots = len(sys.argv) > 3 and sys.argv[3] == '1'
if plots:
    from spark_df_profiling import plot
    plot.start_pool()
import torch  # noqa: E402

import bench  # noqa: E402
from spark_df_profiling import describe  # noqa: E402

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
comm = None
if sharded:
    import socket
    import torch.distributed as dist
    with socket.socket() as sk:
        sk.bind(('127.0.0.1', 0))
        port = sk.getsockname()[1]
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % port, rank=0, world_size=1, device_id=dev)
    from spark_df_profiling.comm import TorchComm
    comm = TorchComm(force_sharded=True)
t = bench.make_c3_shard(rows, 0, 1, dev)
for _ in range(2):
    describe(t, comm=comm, plots=plots)
torch.cuda.synchronize()
t0 = time.perf_counter()
describe(t, comm=comm, plots=plots)
torch.cuda.synchronize()
print('step ms %.2f' % ((time.perf_counter() - t0) * 1e3))
if comm is not None:
    comm.calls.clear()
pr = cProfile.Profile()
pr.enable()
describe(t, comm=comm, plots=plots)
torch.cuda.synchronize()
pr.disable()
if comm is not None:
    print('collectives per step', dict(comm.calls))
st = pstats.Stats(pr)
st.sort_stats('cumulative').print_stats(r'spark_df_profiling|torch/distributed/distributed_c10d|tensor', 45)
st.sort_stats('tottime').print_stats(25)
if sharded:
    import torch.distributed as dist
    dist.destroy_process_group()
