"""Rank communication for the row-sharded engine.

One process per GPU; each rank holds a contiguous row range of every column.
Every statistic resolves through one of three collectives:

* ``allgather``  -- pass-1 states, quantile samples, small candidate sets, top-k
  lists; merged on every rank in rank order (deterministic results);
* ``allreduce_sum`` -- histograms, radix digit histograms, Gram partials, counts
  (int64 sums are exact, so order does not matter);
* ``alltoallv`` -- hash-partitioned distinct keys / (key, count) groups.

`LocalComm` is the single-process identity.  `TorchComm` uses
torch.distributed: backend 'nccl' is RCCL over xGMI on ROCm; 'gloo' is used by
the CPU tests (tensors are moved to the host for the collective); it runs the
same all_to_all_single calls as RCCL, on host copies.  RCCL itself refuses two
ranks on one GPU ("Duplicate GPU detected", tools/rccl_probe.py); a one-rank
nccl group with force_sharded=True runs the same branches on one GPU
(conftest.py starts tests/multirank_worker.py that way).
"""

from __future__ import annotations

from typing import List

import torch


def to_dev(data, dtype, device):
    """A host list / array as a device tensor without a stream sync: staged in
    pinned memory and copied with non_blocking=True (torch.tensor(...,
    device=cuda) from pageable memory synchronises the stream after the copy,
    i.e. waits for every kernel queued before it)."""
    t = torch.as_tensor(data, dtype=dtype)
    if torch.device(device).type != 'cuda':
        return t.to(device)
    return t.pin_memory().to(device, non_blocking=True)


class LocalComm:
    rank = 0
    world = 1
    sharded = False

    def allgather(self, t: torch.Tensor) -> List[torch.Tensor]:
        return [t]

    def allgatherv(self, t: torch.Tensor) -> List[torch.Tensor]:
        return [t]

    def allreduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def allreduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def alltoallv(self, send: torch.Tensor, send_counts: List[int]) -> torch.Tensor:
        assert len(send_counts) == 1
        return send

    def alltoallv_known(self, send: torch.Tensor, send_counts: List[int], recv_counts: List[int]) -> torch.Tensor:
        assert len(send_counts) == 1 and list(send_counts) == list(recv_counts)
        return send

    def alltoallv_known_async(self, send, send_counts, recv_counts):
        return self.alltoallv_known(send, send_counts, recv_counts), _DONE

    def alltoall_counts(self, rows):
        return [list(r) for r in rows]

    def alltoall_counts_dev(self, rows):
        r = rows.cpu().tolist()
        return r, [list(x) for x in r]

    def allgather_object(self, obj, cap=None):
        return [obj]

    def barrier(self):
        pass


class _Done:
    def wait(self):
        pass


_DONE = _Done()


class TorchComm:
    """`sharded` selects the row-sharded code paths (per-round collectives,
    owner exchanges).  It is on whenever world > 1; force_sharded=True (or
    SDP_FORCE_SHARDED=1) turns it on for a one-rank group too, so the RCCL
    branches -- stream-ordered in-place all-reduces, all_to_all_single on
    device tensors, the owner exchanges -- run on a single GPU (RCCL refuses
    two ranks on one device, tools/rccl_probe.py)."""

    def __init__(self, group=None, force_sharded=None):
        import os
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.cpu = self.backend == 'gloo'
        if force_sharded is None:
            force_sharded = os.environ.get('SDP_FORCE_SHARDED', '0') == '1'
        self.sharded = self.world > 1 or bool(force_sharded)
        from collections import Counter
        self.calls = Counter()          # collective -> times issued (tests check the branches ran)

    def _io(self, t):
        return t.cpu() if self.cpu else t

    def allgather(self, t):
        self.calls['allgather'] += 1
        x = self._io(t.contiguous())
        outs = [torch.empty_like(x) for _ in range(self.world)]
        self.dist.all_gather(outs, x, group=self.group)
        return [o.to(t.device) for o in outs]

    def allgatherv(self, t):
        """all_gather of 1-D tensors whose lengths differ per rank."""
        self.calls['allgatherv'] += 1
        n = torch.full((1,), t.numel(), dtype=torch.int64, device=t.device)
        sizes = [int(s.item()) for s in self.allgather(n)]
        m = max(sizes) if sizes else 0
        pad = torch.zeros(m, dtype=t.dtype, device=t.device)
        if t.numel():
            pad[:t.numel()] = t.reshape(-1)
        outs = self.allgather(pad)
        return [o[:s] for o, s in zip(outs, sizes)]

    def allreduce_sum(self, t):
        self.calls['allreduce_sum'] += 1
        x = self._io(t.contiguous()).clone()
        self.dist.all_reduce(x, op=self.dist.ReduceOp.SUM, group=self.group)
        return x.to(t.device)

    def allreduce_sum_(self, t):
        """In-place sum.  With RCCL the collective is ordered on the current
        stream and the host does not wait (device-driven radix rounds)."""
        self.calls['allreduce_sum_'] += 1
        if self.cpu:
            x = t.cpu()
            self.dist.all_reduce(x, op=self.dist.ReduceOp.SUM, group=self.group)
            t.copy_(x)
        else:
            self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return t

    def alltoallv(self, send, send_counts):
        """send is laid out rank-major (send_counts[r] elements for rank r)."""
        self.calls['alltoallv'] += 1
        # gloo runs the same all_to_all_single calls on host copies, so the
        # CPU tests exercise exactly the split logic RCCL sees
        dev = send.device
        counts = self._io(to_dev(send_counts, torch.int64, dev))
        recv_counts = torch.empty_like(counts)
        self.dist.all_to_all_single(recv_counts, counts, group=self.group)
        return self.alltoallv_known(send, send_counts, recv_counts.tolist())

    def alltoallv_known(self, send, send_counts, recv_counts):
        """alltoallv when every rank already knows its receive counts."""
        self.calls['alltoallv_known'] += 1
        dev = send.device
        x = self._io(send.contiguous())
        out = torch.empty(sum(recv_counts), dtype=send.dtype, device=x.device)
        self.dist.all_to_all_single(out, x, output_split_sizes=list(recv_counts),
                                    input_split_sizes=list(send_counts), group=self.group)
        return out.to(dev)

    def alltoallv_known_async(self, send, send_counts, recv_counts):
        """Start alltoallv_known: returns (out, work); `out` holds the result
        after work.wait().  RCCL: the collective runs on its own stream and
        wait() only orders the current stream after it (no host wait), so the
        caller can queue independent kernels meanwhile; `send` must stay
        referenced until then.  gloo: done at once."""
        if self.cpu:
            return self.alltoallv_known(send, send_counts, recv_counts), _DONE
        self.calls['alltoallv_known'] += 1
        out = torch.empty(sum(recv_counts), dtype=send.dtype, device=send.device)
        work = self.dist.all_to_all_single(out, send.contiguous(), output_split_sizes=list(recv_counts),
                                           input_split_sizes=list(send_counts), group=self.group, async_op=True)
        return out, work

    def alltoall_counts(self, rows):
        """rows: k lists of `world` ints (row j, entry r = what this rank sends
        rank r) -> k lists of `world` ints (entry r = what rank r sends this
        rank): every count of an exchange in ONE all-to-all and one readback."""
        self.calls['alltoall_counts'] += 1
        k = len(rows)
        dev = torch.device('cpu') if self.cpu else torch.device('cuda', torch.cuda.current_device())
        send = to_dev(torch.tensor(rows, dtype=torch.int64).t().contiguous(), torch.int64, dev)   # [world, k]
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send, group=self.group)
        r = recv.cpu().tolist()
        return [[r[src][j] for src in range(self.world)] for j in range(k)]

    def alltoall_counts_dev(self, rows):
        """alltoall_counts of counts still on the device (rows: int64 [k, world])
        -> (sent, received), each k lists of `world` ints, with ONE readback of
        both: the sender needs no readback of its own counts before the
        exchange."""
        self.calls['alltoall_counts'] += 1
        k, w = int(rows.shape[0]), self.world
        send = self._io(rows.t().contiguous())                       # [world, k]
        recv = torch.empty_like(send)
        self.dist.all_to_all_single(recv, send, group=self.group)
        both = torch.cat([send.view(-1), recv.view(-1)]).cpu().tolist()
        s, r = both[:w * k], both[w * k:]
        return ([[s[d * k + j] for d in range(w)] for j in range(k)],
                [[r[src * k + j] for src in range(w)] for j in range(k)])

    # bytes of a pickled object that ride the first all-gather round; a larger
    # object on any rank costs a second round sized by the largest
    OBJECT_CAP = 1 << 16

    def allgather_object(self, obj, cap=None):
        """all_gather_object in one tensor collective and ONE readback in the
        common case: every rank sends [size | pickled bytes padded to
        OBJECT_CAP] from pinned memory (no stream sync on the way in); torch's
        all_gather_object pays a pageable upload and two readbacks (sizes, then
        data).  A rank whose payload exceeds the cap makes every rank run a
        second round of the largest size.  `cap` (the same on every rank)
        raises the first round's size for a payload known to be large."""
        import pickle
        import numpy as np
        self.calls['allgather_object'] += 1
        payload = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
        dev = torch.device('cpu') if self.cpu else torch.device('cuda', torch.cuda.current_device())

        def round_(cap):
            buf = np.zeros(8 + cap, dtype=np.uint8)
            buf[:8] = np.frombuffer(np.int64(len(payload)).tobytes(), dtype=np.uint8)
            m = min(cap, len(payload))
            buf[8:8 + m] = np.frombuffer(payload[:m], dtype=np.uint8)
            t = to_dev(buf, torch.uint8, dev)
            outs = [torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(outs, t, group=self.group)
            return torch.stack(outs).cpu().numpy()
        cap0 = max(self.OBJECT_CAP, int(cap or 0))
        got = round_(cap0)
        sizes = [int(np.frombuffer(r[:8].tobytes(), dtype=np.int64)[0]) for r in got]
        if max(sizes) > cap0:
            self.calls['allgather_object_round2'] += 1
            got = round_(max(sizes))
        return [pickle.loads(r[8:8 + sz].tobytes()) for r, sz in zip(got, sizes)]

    def barrier(self):
        self.calls['barrier'] += 1
        self.dist.barrier(group=self.group)
