"""Row-sharded grouping across ranks.

Each rank aggregates its own rows on its GPU (libsdp hash tables), then the
groups are repartitioned by key hash so that every key has exactly one owner
rank (all-to-all), and the owner re-aggregates what it received:

* distinct count  = sum over owners of their group counts (all-reduce);
* value counts    = each owner's top-k by (count desc, key asc), all-gathered
                    and merged on every rank in the same order;
* first rows      = every rank's first k na.drop rows, concatenated in rank order
                    (rank r holds the r-th contiguous row range).

The exchange itself is data movement: the groups are put in owner order by
one libsdp call (sdp_owner_order: owner histogram, scan, stable scatter), the
key bytes packed by sdp_gather_bytes, then all_to_all_single; aggregation runs
in the same HIP kernels as the single-GPU path.
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as nat
from ._native import sdp, ptr
from .comm import to_dev

def _owner_u64(keys: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank of each u64 key (stored as int64): a multiplicative hash."""
    h = keys * -7046029254386353131            # 0x9E3779B97F4A7C15 as int64; wraps
    return ((h >> 40) & 0xFFFFFF) % world


def _table_sel(engine, tab):
    """Entries of the occupied slots of a local table: (indices, count)."""
    slots, counts, cap = tab['slots'], tab['counts'], tab['capacity']
    flags = int(tab['bytes']) | (2 if tab.get('dense') else 0)
    n_local = tab['groups_local'] if 'groups_local' in tab else tab['groups']
    sel = engine._u64(max(n_local, 1))
    nsel = engine._u64(1, zero=True)
    sdp.sdp_table_select(ptr(slots), ptr(counts), cap, flags, 1 if counts is not None else 0,
                         (1 << 64) - 1, ptr(sel), ptr(nsel), max(n_local, 1), engine._s())
    return sel, int(nsel.item())


def _owner_order(engine, keys, sel, counts, n, bcol=None, with_counts=True):
    """sdp_owner_order: the groups owner-major (stable within an owner), one
    libsdp call.  Returns the output tensors and per = [2, world] (groups,
    key bytes) per owner, still on the device."""
    world = engine.comm.world
    dev = engine.device
    out = {'per': torch.empty(2 * world, dtype=torch.int64, device=dev)}
    m = max(n, 1)
    if bcol is None:
        out['keys'] = torch.empty(m, dtype=torch.int64, device=dev)
        out['counts'] = torch.empty(m, dtype=torch.int64, device=dev) if with_counts else None
    else:
        for k in ('starts', 'lens'):
            out[k] = torch.empty(m, dtype=torch.int64, device=dev)
        out['meta'] = torch.empty(2 * m, dtype=torch.int64, device=dev)
        out['offs'] = torch.empty(n + 1, dtype=torch.int64, device=dev)
    wb = sdp.sdp_owner_order_workspace_bytes(n, world)
    work = engine._bytes(max(wb, 16))
    sdp.sdp_owner_order(ptr(keys), ptr(sel) if sel is not None else None,
                        ptr(counts) if counts is not None else None, n, world,
                        ctypes.byref(bcol) if bcol is not None else None,
                        ptr(out['keys']) if bcol is None else None,
                        ptr(out['counts']) if bcol is None and out['counts'] is not None else None,
                        *[ptr(out[k]) if bcol is not None else None for k in ('starts', 'lens', 'meta', 'offs')],
                        ptr(out['per']), ptr(work), wb, engine._s())
    for k in list(out):
        if k not in ('per', 'offs') and out[k] is not None:
            out[k] = out[k][:n] if k != 'meta' else out[k][:2 * n]
    out['_work'] = work
    return out


def exchange_fixed_groups(engine, tab, with_counts):
    comm = engine.comm
    world = comm.world
    sel, m = _table_sel(engine, tab)
    oo = _owner_order(engine, tab['slots'], sel, tab['counts'] if with_counts else None, m,
                      with_counts=with_counts)
    sent, got = comm.alltoall_counts_dev(oo['per'][:world].view(1, world))
    send, recv = sent[0], got[0]
    rkeys = comm.alltoallv_known(oo['keys'], send, recv)
    rcnt = None
    if with_counts:
        rcnt = comm.alltoallv_known(oo['counts'], send, recv)
    # owner table over the received keys (they are already order-preserving
    # u64 keys: a U64 column hashes them unchanged)
    from .columns import DeviceColumn
    col = DeviceColumn('_exchange', 'bigint', int(rkeys.numel()), 'fixed', nat.U64)
    col.values = rkeys if rkeys.numel() else torch.zeros(2, dtype=torch.int64, device=engine.device)
    local = engine._distinct_fixed_table(col, with_counts=with_counts, row_counts=rcnt, exchanged=True)
    side = to_dev([tab['max_key_rows'], tab['rows'], local['groups'] - (1 if local['max_key_rows'] else 0)],
                  torch.int64, engine.device)
    tot = comm.allreduce_sum(side).tolist()
    max_rows, rows, owner_groups = int(tot[0]), int(tot[1]), int(tot[2])
    local['groups_local'] = local['groups'] - (1 if local['max_key_rows'] else 0)
    local['max_key_rows'] = max_rows if comm.rank == 0 else 0
    local['groups'] = owner_groups + (1 if max_rows else 0)
    local['rows'] = rows
    local['sharded'] = True
    return local


def exchange_bytes_groups(engine, tab):
    """exchange_bytes_groups_batch of one rank-local table."""
    return exchange_bytes_groups_batch(engine, [tab])[0]


def exchange_bytes_groups_batch(engine, tabs):
    """Re-partition every rank's byte-key groups of several columns by key
    hash: each group's (length, count) and its key bytes go to the owner rank,
    which re-aggregates them in a global table.  The columns share their host
    round trips: ONE all-to-all + readback of every column's per-owner group
    and byte counts (sent and received together), ONE readback of every owner
    table's statistics with the all-reduced totals (round 2 paid four per
    column, round 5 three per batch)."""
    comm = engine.comm
    world = comm.world
    if not tabs:
        return []
    preps, pers = [], []
    for tab in tabs:
        col = tab['col']
        if tab.get('dense'):
            # partitioned groups are already packed: every entry is a group
            sel, m = None, int(tab['groups_local'])
        else:
            sel, m = _table_sel(engine, tab)
        bc = col.sdp_bytes()
        oo = _owner_order(engine, tab['slots'], sel, tab['counts'], m, bcol=bc)
        pers.append(oo['per'].view(2, world))
        preps.append((tab, col, oo))
    # every column's per-owner group and byte counts: sent and received in ONE
    # all-to-all and one readback
    sent, recv = comm.alltoall_counts_dev(torch.stack(pers).view(-1, world))
    allper = [(sent[2 * j], sent[2 * j + 1]) for j in range(len(preps))]
    payloads = []
    for (tab, col, oo), (send_groups, send_bytes) in zip(preps, allper):
        # key bytes of every group, owner-major, packed by one native gather
        tot = sum(send_bytes)
        payload = torch.empty(max(tot, 1), dtype=torch.uint8, device=engine.device)[:tot]
        if tot:
            sdp.sdp_gather_bytes(ptr(col.data), ptr(oo['starts']), ptr(oo['lens']), ptr(oo['offs']),
                                 oo['lens'].numel(), ptr(payload), engine._s())
        payloads.append(payload)
    launched = []
    for j, ((tab, col, oo), (send_groups, send_bytes), payload) in enumerate(zip(preps, allper, payloads)):
        recv_groups, recv_bytes = recv[2 * j], recv[2 * j + 1]
        # (length, count) pairs in one exchange, the key bytes in a second
        meta = oo['meta']
        rmeta = comm.alltoallv_known(meta, [2 * g for g in send_groups], [2 * g for g in recv_groups]).view(-1, 2)
        rbytes = comm.alltoallv_known(payload.contiguous(), send_bytes, recv_bytes)
        rlens, rcnt = rmeta[:, 0].contiguous(), rmeta[:, 1].contiguous()
        from .columns import DeviceColumn
        n = int(rlens.numel())
        rc = DeviceColumn('_exchange', col.spark_type, n, 'bytes', decimal_scale=col.decimal_scale)
        offs = torch.zeros(n + 1, dtype=torch.int64, device=engine.device)
        if n:
            torch.cumsum(rlens, 0, out=offs[1:])
        rc.offsets = offs
        rc.offset_width = 8
        data = torch.zeros(int(rbytes.numel()) + 16, dtype=torch.uint8, device=engine.device)
        data[:rbytes.numel()] = rbytes
        rc.data = data
        launched.append((tab, rc, engine.bytes_table_launch(rc, row_counts=rcnt)))
    # the owner tables' statistics and the (rows, groups) totals over the ranks
    # (summed on the device) in ONE readback
    stats = torch.cat([lt[2]['stats'] for lt in launched]).view(-1, 4)
    rows = to_dev([tab['rows'] for tab, _, _ in launched], torch.int64, engine.device)
    tot = comm.allreduce_sum(torch.stack([rows, stats[:, 0]], 1).reshape(-1))
    host = engine._host_u64(torch.cat([stats.reshape(-1), tot]))
    st, t = host[:stats.numel()], host[stats.numel():]
    locals_ = []
    for j, (tab, rc, pend) in enumerate(launched):
        local = engine.bytes_table_finish(pend, st[4 * j:4 * j + 4], rc)
        local['src_col'] = rc
        local['col'] = rc
        locals_.append(local)
    for j, local in enumerate(locals_):
        local['groups_local'] = local['groups']
        local['groups'] = int(t[2 * j + 1])
        local['rows'] = int(t[2 * j])
        local['sharded'] = True
    return locals_


def merge_topk(comm, pairs, k):
    """Global top-k from every rank's local top-k list of (value, count)."""
    if not comm.sharded:
        return pairs[:k]
    allp = comm.allgather_object(pairs)
    merged = [p for part in allp for p in part]
    merged.sort(key=lambda vc: (-vc[1], _sortable(vc[0])))
    return merged[:k]


def merge_topk_batch(comm, pairs_list, k):
    """merge_topk of several columns with ONE all-gather (each all_gather_object
    is two host round trips)."""
    if not comm.sharded:
        return [pairs[:k] for pairs in pairs_list]
    allp = comm.allgather_object(list(pairs_list))
    out = []
    for j in range(len(pairs_list)):
        merged = [p for part in allp for p in part[j]]
        merged.sort(key=lambda vc: (-vc[1], _sortable(vc[0])))
        out.append(merged[:k])
    return out


def _sortable(v):
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    if isinstance(v, (np.integer,)):
        return int(v)
    if isinstance(v, (np.floating,)):
        return float(v)
    return v


def merge_first_rows(comm, values, k):
    if not comm.sharded:
        return values[:k]
    allv = comm.allgather_object(values)
    out = []
    for part in allv:
        out.extend(part)
        if len(out) >= k:
            break
    return out[:k]
