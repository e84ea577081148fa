"""Debug: group_sharded on a tiny column over 2 gloo ranks (one GPU)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'spark-df-profiling_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)
import numpy as np, pyarrow as pa, torch, torch.distributed as dist
rank = int(os.environ['RANK']); world = int(os.environ['WORLD_SIZE'])
dev = torch.device('cuda', 0); torch.cuda.set_device(dev)
dist.init_process_group('gloo')
from spark_df_profiling.columns import DeviceTable
from spark_df_profiling.comm import TorchComm
from spark_df_profiling.engine import Engine
import spark_df_profiling.engine as E
vals = [50, 50, -10, 0, 0, 5, 15, -3, None]
t = pa.table({'x': pa.array(vals, pa.int64())})
full = DeviceTable.from_arrow(t, dev)
per = 0 if int(sys.argv[1]) == 0 else 16
sh = full.slice_rows(0, per) if rank == 0 else full.slice_rows(per, t.num_rows) if per < t.num_rows else full.slice_rows(per, per)
e = Engine(device=dev, comm=TorchComm())
orig = e._host_u64
def hu(x):
    r = orig(x); print('rank', rank, 'host_u64', r[:8], flush=True); return r
e._host_u64 = hu
tab = e.group_sharded(sh.columns[0])
print('rank', rank, 'n', sh.columns[0].length, 'groups', tab['groups'] if tab else None, flush=True)
dist.destroy_process_group()
