"""Row-sharded grouping across ranks.

Each rank aggregates its own rows on its GPU (libsdp hash tables), then the
groups are repartitioned by key hash so that every key has exactly one owner
rank (all-to-all), and the owner re-aggregates what it received:

* distinct count  = sum over owners of their group counts (all-reduce);
* value counts    = each owner's top-k by (count desc, key asc), all-gathered
                    and merged on every rank in the same order;
* first rows      = every rank's first k na.drop rows, concatenated in rank order
                    (rank r holds the r-th contiguous row range).

The exchange itself is data movement (gather by owner, all_to_all_single);
aggregation runs in the same HIP kernels as the single-GPU path.
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native as nat
from ._native import sdp, ptr
from .comm import to_dev

MASK40 = (1 << 40) - 1


def _owner_u64(keys: torch.Tensor, world: int) -> torch.Tensor:
    """Owner rank of each u64 key (stored as int64): a multiplicative hash."""
    h = keys * -7046029254386353131            # 0x9E3779B97F4A7C15 as int64; wraps
    return ((h >> 40) & 0xFFFFFF) % world


def _table_groups(engine, tab):
    """Dense (keys, counts) of a local table (all occupied slots)."""
    slots, counts, cap = tab['slots'], tab['counts'], tab['capacity']
    flags = int(tab['bytes']) | (2 if tab.get('dense') else 0)
    n_local = tab['groups_local'] if 'groups_local' in tab else tab['groups']
    sel = engine._u64(max(n_local, 1))
    nsel = engine._u64(1, zero=True)
    sdp.sdp_table_select(ptr(slots), ptr(counts), cap, flags, 1 if counts is not None else 0,
                         (1 << 64) - 1, ptr(sel), ptr(nsel), max(n_local, 1), engine._s())
    m = int(nsel.item())
    sel = sel[:m]
    keys = slots[sel]
    cnt = counts[sel] if counts is not None else None
    return keys, cnt


def exchange_fixed_groups(engine, tab, with_counts):
    comm = engine.comm
    world = comm.world
    keys, cnt = _table_groups(engine, tab)
    owner = _owner_u64(keys, world)
    order = _owner_order(owner, world)
    keys = keys[order]
    bounds = torch.searchsorted(owner[order], torch.arange(world + 1, dtype=owner.dtype, device=engine.device))
    send = (bounds[1:] - bounds[:-1]).tolist()
    recv = comm.alltoall_counts([send])[0]
    rkeys = comm.alltoallv_known(keys.contiguous(), send, recv)
    rcnt = None
    if with_counts:
        rcnt = comm.alltoallv_known(cnt[order].contiguous(), send, recv)
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


def _owner_order(owner, world):
    """Stable order of the groups by owner rank: a radix sort of 1- or 2-byte
    keys (one or two passes) instead of an int64 argsort."""
    key = owner.to(torch.uint8 if world <= 256 else torch.int16)
    return torch.sort(key, stable=True)[1]


def exchange_bytes_groups(engine, tab):
    """exchange_bytes_groups_batch of one rank-local table."""
    return exchange_bytes_groups_batch(engine, [tab])[0]


def exchange_bytes_groups_batch(engine, tabs):
    """Re-partition every rank's byte-key groups of several columns by key
    hash: each group's (length, count) and its key bytes go to the owner rank,
    which re-aggregates them in a global table.  The columns share their host
    round trips: ONE readback of every column's per-owner group and byte
    counts, ONE all-to-all of every count of every exchange, ONE readback of
    every owner table's statistics, ONE all-reduce of the totals (round 2 paid
    these four per column)."""
    comm = engine.comm
    world = comm.world
    if not tabs:
        return []
    preps, pers = [], []
    for tab in tabs:
        col = tab['col']
        if tab.get('dense'):
            # partitioned groups are already packed: every entry is a group
            m = int(tab['groups_local'])
            slots, cnt = tab['slots'][:m], tab['counts'][:m]
        else:
            slots, cnt = _table_groups(engine, tab)
        rows = (slots & MASK40) - 1
        owner = ((slots >> 40) & 0xFFFFFF) % world
        order = _owner_order(owner, world)
        rows, cnt, owner = rows[order], cnt[order], owner[order]
        if col.fixed_width:
            starts = rows * col.fixed_width
            lens = torch.full_like(rows, col.fixed_width)
        else:
            o = col.offsets.to(torch.int64)
            starts = o[rows]
            lens = o[rows + 1] - starts
        # groups and key bytes per owner from the owner-sorted order: range
        # bounds by searchsorted and a prefix sum of the lengths (a scatter_add
        # into `world` counters serialised every group's atomic on a few
        # addresses: 4.2 ms per 1.25e8-row step, profiles/r03q_*)
        bounds = torch.searchsorted(owner, torch.arange(world + 1, dtype=owner.dtype, device=engine.device))
        pref = torch.zeros(lens.numel() + 1, dtype=torch.int64, device=engine.device)
        torch.cumsum(lens, 0, out=pref[1:])
        per = torch.stack([bounds[1:] - bounds[:-1], pref[bounds[1:]] - pref[bounds[:-1]]])
        pers.append(per)
        preps.append((tab, col, starts, lens, cnt, pref[:-1]))
    allper = torch.stack(pers).cpu().tolist()                     # [column][groups | bytes][owner]
    payloads = []
    for (tab, col, starts, lens, cnt, offs), (send_groups, send_bytes) in zip(preps, allper):
        # key bytes of every group, owner-major, packed by one native gather
        tot = sum(send_bytes)
        payload = torch.empty(max(tot, 1), dtype=torch.uint8, device=engine.device)[:tot]
        if tot:
            sdp.sdp_gather_bytes(ptr(col.data), ptr(starts.contiguous()), ptr(lens.contiguous()), ptr(offs),
                                 lens.numel(), ptr(payload), engine._s())
        payloads.append(payload)
    recv = comm.alltoall_counts([row for pr in allper for row in pr])
    launched = []
    for j, ((tab, col, starts, lens, cnt, _), (send_groups, send_bytes), payload) in enumerate(zip(preps, allper,
                                                                                                  payloads)):
        recv_groups, recv_bytes = recv[2 * j], recv[2 * j + 1]
        # (length, count) pairs in one exchange, the key bytes in a second
        meta = torch.stack([lens, cnt], 1).contiguous().view(-1)
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
    st = engine._host_u64(torch.cat([lt[2]['stats'] for lt in launched]))
    locals_, sides = [], []
    for j, (tab, rc, pend) in enumerate(launched):
        local = engine.bytes_table_finish(pend, st[4 * j:4 * j + 4], rc)
        local['src_col'] = rc
        local['col'] = rc
        locals_.append(local)
        sides += [tab['rows'], local['groups']]
    t = comm.allreduce_sum(to_dev(sides, torch.int64, engine.device)).tolist()
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
