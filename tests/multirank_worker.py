"""Row-sharded describe() on N ranks vs the oracle on the whole table.

Run with one GPU per rank over RCCL, or several ranks sharing one GPU over gloo:
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29511 tests/multirank_worker.py [nccl|gloo] [table,...]
tests/test_gpu_multirank.py runs it (2 gloo ranks on the one GPU of the box),
started by conftest.py before the test process initialises the GPU.
"""
import os
import sys

os.environ.setdefault('SDP_PLOT_WORKERS', '0')      # render inline (no pool in this check)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # repo root
for p in (ROOT, os.path.join(ROOT, 'spark-df-profiling_amd'), os.path.join(ROOT, 'tests')):
    sys.path.insert(0, p)

import pyarrow as pa
import torch
import torch.distributed as dist

import datagen
from compare import assert_describe_equal


def _check_gk(comm, rank, world, dev):
    """quantile_mode='gk' on a row-sharded float column: rank r's rows form
    Spark partitions r*k .. r*k+k-1 (k = 2 per rank), so the answer is
    percentile_approx over those partitions in rank-major order."""
    import numpy as np
    from spark_df_profiling import describe
    from spark_df_profiling.columns import DeviceTable
    rng = np.random.default_rng(23)
    n = 70_001
    x = rng.lognormal(0.0, 1.5, n)
    x[rng.random(n) < 0.01] = np.nan
    x[::97] = 1.0                                    # a heavy value
    valid = rng.random(n) > 0.02
    t = pa.table({'x': pa.array(x, mask=~valid)})
    full = DeviceTable.from_arrow(t, dev)
    per = (n // world) // 16 * 16
    bounds = [(r * per, n if r == world - 1 else (r + 1) * per) for r in range(world)]
    start, stop = bounds[rank]
    k = 2
    got = describe(full.slice_rows(start, stop), comm=comm, plots=False, quantile_mode='gk',
                   spark_partitions=k * world)
    if rank != 0:
        return 0
    from oracle import gk
    parts = []
    for a, b in bounds:
        parts += gk.split_rows(x[a:b], valid[a:b], k)
    probs = [0.05, 0.25, 0.5, 0.75, 0.95]
    want = gk.percentile_approx(parts, probs)
    v = got['variables']
    bad = [(p, v.loc['x', '%d%%' % int(p * 100)], w) for p, w in zip(probs, want)
           if v.loc['x', '%d%%' % int(p * 100)] != w]
    if bad:
        print('[gk] MISMATCH world=%d %s' % (world, bad), flush=True)
        return 1
    print('[gk] OK world=%d' % world, flush=True)
    return 0


def main():
    backend = sys.argv[1] if len(sys.argv) > 1 else 'gloo'
    rank = int(os.environ['RANK'])
    world = int(os.environ['WORLD_SIZE'])
    local = int(os.environ.get('LOCAL_RANK', '0'))
    ngpu = torch.cuda.device_count()
    dev = torch.device('cuda', local % ngpu)
    torch.cuda.set_device(dev)
    if backend == 'nccl':
        dist.init_process_group('nccl', device_id=dev)
    else:
        dist.init_process_group('gloo')
    from spark_df_profiling import describe
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.comm import TorchComm
    comm = TorchComm()
    tables = {
        'demo': datagen.demo_like_table(60_000),
        'numeric': datagen.numeric_table(40_000),
        'numeric_big': datagen.numeric_table(300_001, seed=11),
        'categorical': datagen.categorical_table(30_000),
        # >= 64 K rows per rank: byte columns take the local partitioning path
        'categorical_big': datagen.categorical_table(240_000, seed=9, card=(100, 100_000)),
        'dates': datagen.date_table(20_000),
        'corr': datagen.corr_table(20_000),
        'legacy': datagen.legacy_table(),
        # sorted columns across rank boundaries (equal keys on both sides of a boundary)
        'sorted': datagen.sorted_table(200_003),
    }
    if 'c3' in (sys.argv[2].split(',') if len(sys.argv) > 2 else []):
        import bench
        # the bench generator at 4 M rows, made on the device (rank-independent: the
        # whole table is built on every rank and sliced like the others)
        tables['c3'] = bench.shard_to_arrow(bench.make_c3_shard(4_000_000, 0, 1, dev))
    only = sys.argv[2].split(',') if len(sys.argv) > 2 else None
    failures = 0
    for name, t in tables.items():
        if only and name not in only:
            continue
        full = DeviceTable.from_arrow(t, dev)
        n = t.num_rows
        per = (n // world) // 16 * 16
        start = rank * per
        stop = n if rank == world - 1 else start + per
        shard = full.slice_rows(start, stop)
        plots = name == 'numeric'
        got = describe(shard, comm=comm, plots=plots)
        if plots:
            # each rank rendered its own columns; every rank must hold all images
            v = got['variables']
            num = v[v['type'] == 'NUM']
            bad = [c for c in num.index if not str(num.loc[c, 'histogram']).startswith('data:image/png')
                   or not str(num.loc[c, 'mini_histogram']).startswith('data:image/png')]
            if bad:
                failures += 1
                print('[%s] rank %d missing images for %s' % (name, rank, bad), flush=True)
        if rank == 0:
            import oracle
            if t.num_rows > 1_000_000:
                from oracle import fast
                want = fast.describe(t)
            else:
                want = oracle.describe(t)
            try:
                assert_describe_equal(got, want)
                print('[%s] OK world=%d' % (name, world), flush=True)
            except AssertionError as e:
                failures += 1
                print('[%s] MISMATCH world=%d\n%s' % (name, world, e), flush=True)
    if not only or 'gk' in only:
        failures += _check_gk(comm, rank, world, dev)
    dist.barrier()
    dist.destroy_process_group()
    if rank == 0:
        # the collectives the sharded path issued (SDP_REQUIRE_CALLS: each must have run)
        print('[calls] backend=%s sharded=%s %s' % (comm.backend, comm.sharded, dict(comm.calls)), flush=True)
        need = [c for c in os.environ.get('SDP_REQUIRE_CALLS', '').split(',') if c]
        missing = [c for c in need if not comm.calls.get(c)]
        if missing:
            failures += 1
            print('[calls] MISSING %s' % missing, flush=True)
        print('MULTIRANK %s failures=%d' % ('OK' if not failures else 'FAILED', failures), flush=True)
    if failures:
        sys.exit(1)


if __name__ == '__main__':
    main()
