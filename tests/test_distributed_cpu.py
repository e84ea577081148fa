"""world_size-2 gloo tests of the rank-merge logic (CPU only, no kernels)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from spark_df_profiling.comm import TorchComm
        from spark_df_profiling.distributed import merge_topk, merge_first_rows, _owner_u64
        from spark_df_profiling import engine as eng
        from spark_df_profiling import _native as nat
        comm = TorchComm()
        out = {}
        # allgather / allgatherv / allreduce
        t = torch.tensor([rank + 1.0, 10.0 * rank], dtype=torch.float64)
        out['allgather'] = [x.tolist() for x in comm.allgather(t)]
        v = torch.arange(rank + 2, dtype=torch.int64)
        out['allgatherv'] = [x.tolist() for x in comm.allgatherv(v)]
        out['allreduce'] = comm.allreduce_sum(torch.tensor([rank + 1], dtype=torch.int64)).tolist()
        # in-place all-reduce of a [Q, 2048] digit-histogram block (sharded radix select)
        h = torch.zeros(3 * 2048, dtype=torch.int64)
        h[rank * 2048 + 7] = 5
        h[2 * 2048 + 11] = rank + 1
        r_ = comm.allreduce_sum_(h)
        out['allreduce_'] = (r_ is h, int(h[7]), int(h[2048 + 7]), int(h[2 * 2048 + 11]), int(h.sum()))
        # histogram images: every rank ends with every rank's strings
        imgs = {'c%d' % rank: ('h%d' % rank, 'm%d' % rank)}
        for part in comm.allgather_object(dict(imgs)):
            imgs.update(part)
        out['images'] = sorted(imgs.items())
        # an object beyond the one-round cap on one rank: the second round
        big = {'rank': rank, 'blob': bytes([rank]) * (comm.OBJECT_CAP * 2 if rank == 1 else 10)}
        out['big'] = [(o['rank'], len(o['blob']), o['blob'][:1]) for o in comm.allgather_object(big)]
        r2 = comm.calls['allgather_object_round2']
        # the same object with a cap hint every rank agrees on: one round
        out['big_cap'] = [len(o['blob']) for o in comm.allgather_object(big, cap=4 * comm.OBJECT_CAP)]
        out['rounds2'] = (r2, comm.calls['allgather_object_round2'])
        # alltoallv (all_to_all_single, as on RCCL): rank r sends (r*10 + d) repeated d+1 times to rank d
        send = torch.cat([torch.full((d + 1,), rank * 10 + d, dtype=torch.int64) for d in range(world)])
        out['alltoallv'] = comm.alltoallv(send, [d + 1 for d in range(world)]).tolist()
        # per-owner counts still on the device: sent and received with one readback
        rows = torch.tensor([[rank * 100 + j * 10 + d for d in range(world)] for j in range(3)], dtype=torch.int64)
        out['a2ac'] = (comm.alltoall_counts_dev(rows), comm.alltoall_counts(rows.tolist()))
        # top-k merge: (count desc, key asc), deterministic on every rank
        local = [('b%d' % rank, 5), ('a', 3 + rank), ('z%d' % rank, 1)]
        out['topk'] = merge_topk(comm, local, 4)
        out['first'] = merge_first_rows(comm, ['r%d_%d' % (rank, i) for i in range(3)], 4)
        # pass-1 states merged in rank order on every rank
        e = eng.Engine(device='cpu', comm=comm)
        p = nat.SdpPass1Result()
        p.count = 10 + rank
        p.n_valid = 11 + rank
        p.isum = 2 ** 62
        p.imin, p.imax = -rank, rank
        p.dmin, p.dmax = float(-rank), float(rank)
        p.s1_hi, p.s2 = 1.0 + rank, 2.0
        p.w_gt[0] = rank
        m = e.merge_pass1(p)
        out['p1'] = (m['count'], m['n_valid'], m['isum'], m['imin'], m['imax'], m['s1'], m['w_gt'][0])
        out['owner'] = _owner_u64(torch.arange(1000, dtype=torch.int64), world).bincount(minlength=world).tolist()
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_two_rank_merges():
    world = 2
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        o = res[r]
        assert o['allgather'] == [[1.0, 0.0], [2.0, 10.0]]
        assert o['allgatherv'] == [[0, 1], [0, 1, 2]]
        assert o['allreduce'] == [3]
        assert o['allreduce_'] == (True, 5, 5, 3, 13)
        assert o['images'] == [('c0', ('h0', 'm0')), ('c1', ('h1', 'm1'))]
        from spark_df_profiling.comm import TorchComm
        assert o['big'] == [(0, 10, b'\x00'), (1, 2 * TorchComm.OBJECT_CAP, b'\x01')]
        assert o['big_cap'] == [10, 2 * TorchComm.OBJECT_CAP]
        assert o['rounds2'] == (1, 1)
        want = []
        for src in range(world):
            want += [src * 10 + r] * (r + 1)
        assert o['alltoallv'] == want
        sent, got = o['a2ac'][0]
        assert sent == [[r * 100 + j * 10 + d for d in range(world)] for j in range(3)]
        assert got == [[src * 100 + j * 10 + r for src in range(world)] for j in range(3)] == o['a2ac'][1]
        assert o['topk'] == [('b0', 5), ('b1', 5), ('a', 4), ('a', 3)]
        assert o['first'] == ['r0_0', 'r0_1', 'r0_2', 'r1_0']
        assert o['p1'] == (21, 23, 2 ** 63 - 2 ** 64, -1, 1, 3.0, 1)
        assert sum(o['owner']) == 1000 and min(o['owner']) > 350
    same = {k: v for k, v in res[0].items() if k not in ('alltoallv', 'a2ac')}
    assert same == {k: v for k, v in res[1].items() if k not in ('alltoallv', 'a2ac')}
