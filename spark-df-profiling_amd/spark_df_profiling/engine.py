"""Host orchestration of the HIP kernels for one column (and the Pearson matrix).

Everything that touches rows runs in libsdp.so on the GPU; this module only
sizes buffers, launches, reads back the small result structs, merges per-rank
states in rank order and applies the reference's scalar formulas (the
driver-side arithmetic of describe.py: range, iqr, cv, thresholds, edges).

Reference call sites replaced (all /root/reference/spark_df_profiling/):
  describe.py:143   countDistinct            -> distinct_fixed / value_counts_*
  describe.py:144   na.drop().count          -> pass1.count / table stats
  describe.py:193-201 agg(mean..sum)         -> pass1 + moments()
  describe.py:203-208 percentile(_approx)    -> plan + pass1 windows + select_kth
  describe.py:215-223 mad, zeros, outliers   -> pass1.n_zero, pass2
  describe.py:38-63  generate_hist_data      -> hist_edges() + pass2
  describe.py:233    date min/max            -> pass1 (no windows)
  describe.py:250-271 categorical groupBy    -> value_counts_* + topk()
  describe.py:276,:282 limit(1)/limit(50)    -> first_rows()
  utils.py:20-36    corr_matrix              -> rowmask + gram()
"""

from __future__ import annotations

import ctypes
import os
import math
from fractions import Fraction
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from . import _native as nat
from ._native import sdp, ptr
from .comm import LocalComm, to_dev
from .columns import DeviceColumn, decimal_from_key

PROBS = (0.05, 0.25, 0.5, 0.75, 0.95)          # describe.py:207
SAMPLE_TOTAL = 16384
SAMPLE2_TOTAL = 131072        # second sample narrowing the quantile windows (sdp_quantile_refine_batch)
# third sample narrowing them again (its in-window keys, ~4 % of it, must fit
# the refine kernel's 16 K-key LDS sort; 0 disables)
SAMPLE3_TOTAL = int(os.environ.get('SDP_SAMPLE3', 360448))
SORT_MAX = 16384
GSORT_MAX = nat.GSORT_MAX          # (sdp.h SDP_GSORT_MAX, checked at load)
TOPK = 50                                       # describe.py:259
EMPTY64 = 0xFFFFFFFFFFFFFFFF
U64 = (1 << 64) - 1
PART_SAMPLE = nat.PART_SAMPLE      # rows sampled for heavy keys (sdp_part_sample; SDP_PART_SAMPLE)
# byte columns: up to HEAVY_MAX_REC heavy keys need a larger sample to be seen
# HEAVY_MIN times (zipf(1.1) over 1e8 labels: the 1024th key holds ~6e-5 of the rows)
PART_SAMPLE_BYTES = nat.PART_SAMPLE_BYTES
HEAVY_MIN = nat.HEAVY_MIN          # sample occurrences that make a key heavy
# level-2 records per workgroup chunk: each chunk pays its header and bucket
# offsets before its first tile (131072 vs 65536: f64 level-2 scatter 4.4-4.7
# -> 4.1-4.3 ms per 1e9 records; 262144 loses on skewed columns,
# profiles/r04z_part_chunk_ab.log)
PART_CHUNK = nat.PART_CHUNK
# byte columns: strings read once into compacted records, then a record scatter
# (columns too short for two levels, b1 = 0, take the count + scatter row kernels)
BYTES_ONE_READ = True
# pass 1 with inclusive quantile windows where the plan allows (SDP_PASS1_EXCL=1: never, for A/B runs)
PASS1_INCLUSIVE = os.environ.get('SDP_PASS1_EXCL', '0') != '1'
# SDP_PASS1_BATCH=0: one sdp_pass1 launch per column instead of one sdp_pass1_batch per dtype
PASS1_BATCH = os.environ.get('SDP_PASS1_BATCH', '1') != '0'
# SDP_BITS32=0: 32-bit key spaces take the 64-bit partitioning path too (A/B runs)
BITS32 = os.environ.get('SDP_BITS32', '1') != '0'
# SDP_PASS2_BATCH=0: one sdp_pass2_count launch per column on wide tables too
PASS2_BATCH = os.environ.get('SDP_PASS2_BATCH', '1') != '0'
# level 2 into blocks, one workgroup per level-1 bucket, no count pass
# (sdp_part_l2_blocks, round 6; its illegal accesses in r06b were a
# sign-extended readfirstlane pointer, fixed in sdp_common.h's uniform_u64;
# bounds-checked build clean, profiles/r06h_*).  SDP_L2_BLOCKS=0: the counted
# exact-offset level 2 (sdp_part_recs phase 0 + 1) for A/B runs
L2_BLOCKS = os.environ.get('SDP_L2_BLOCKS', '1') != '0'
L2_BLOCK = nat.L2_BLOCK
DEBUG_BOUNDS = os.environ.get('SDP_DEBUG_BOUNDS', '') == '1'      # a tools/debug_bounds.sh library is loaded
CAND_FULL_BUDGET = 1 << 30   # bytes of room-for-every-row candidate slots per pass-1 batch

# Test knob for the quantile edge paths (never set in production):
#   'overflow' -- one candidate slot per wave segment, so every window that
#                 receives candidates overflows (w_overflow) and its ranks take
#                 the exact whole-column select;
#   'miss'     -- every planned window is narrowed to its lower bound, so ranks
#                 outside the bound's ties miss the windows and fall back.
import os as _os
DEBUG_QUANTILE = _os.environ.get('SDP_DEBUG_QUANTILE', '')


def _u(x):
    return int(x) & U64


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


DTYPE_NAME = {nat.I8: 'i8', nat.I16: 'i16', nat.I32: 'i32', nat.I64: 'i64', nat.U8: 'u8', nat.U16: 'u16',
              nat.U32: 'u32', nat.U64: 'u64', nat.F32: 'f32', nat.F64: 'f64', nat.BOOL: 'bool'}


def col_read_bytes(col):
    """Compulsory bytes of one read of a column: values (or offsets + string
    bytes) plus the validity bit."""
    n = col.length
    vb = n / 8.0 if col.validity is not None else 0.0
    if col.kind == 'bytes':
        if col.fixed_width:
            return n * col.fixed_width + vb
        return n * col.offset_width + max(0, col.data.numel() - 16) + vb
    if col.kind != 'fixed':
        return vb
    return n * nat.ELEM_SIZE.get(col.dtype, 8) + vb


def _label(col, stage=''):
    base = 'bytes' if col.kind == 'bytes' else DTYPE_NAME.get(col.dtype, 'fixed')
    return base + ('/' + stage if stage else '')


def inv_mix64(x):
    """Inverse of mix64 (sdp_common.h), so a fixed key is recovered from its record."""
    x ^= x >> 32
    x = (x * 0xCFEE444D8B59A89B) & U64
    return x ^ (x >> 32)


def _next_pow2(x):
    return 1 << max(10, int(x - 1).bit_length())


def key_to_float(k: int) -> float:
    k = _u(k)
    b = (k & 0x7FFFFFFFFFFFFFFF) if (k >> 63) else (~k & U64)
    return float(np.array([b], dtype=np.uint64).view(np.float64)[0])


def key_to_int(k: int) -> int:
    v = _u(k) ^ (1 << 63)
    return v - (1 << 64) if v >= (1 << 63) else v


def spark_percentile_approx_rank(n, p, relative_error=1e-4):
    """1-based rank returned for float columns."""
    if p <= relative_error:
        return 1
    if p >= 1 - relative_error:
        return n
    return min(max(int(math.ceil(p * n)), 1), n)


def hist_edges(minim, maxim, bins):
    """describe.py:40-45: edges by accumulated addition, last popped."""
    num_range = maxim - minim
    bin_width = num_range / float(bins)
    left_edges = [minim]
    for _bin in range(bins):
        left_edges = left_edges + [left_edges[-1] + bin_width]
    left_edges.pop()
    if len(left_edges) < 2:
        raise IndexError('list index out of range')     # describe.py:46 with bins=1
    return left_edges, bin_width


@dataclass
class NumericStats:
    count: int
    n_valid: int
    n_nan: int
    n_zero: int
    min: float
    max: float
    sum: float
    mean: float
    variance: float
    std: float
    skewness: float
    kurtosis: float
    quantiles: Dict[float, float] = field(default_factory=dict)
    mad: float = float('nan')
    hist_counts: Optional[np.ndarray] = None
    edges: Optional[list] = None
    width: float = float('nan')
    high_idx: int = 0
    low_idx: int = 0
    thresholds: tuple = ()
    fallback_used: bool = False
    error: Optional[Exception] = None      # raised when describe_1d reaches the column


class Engine:
    """Kernel driver for one device (and one rank of a sharded table)."""

    def __init__(self, device=None, comm=None, stream=None):
        self.device = torch.device(device or 'cuda')
        self.comm = comm or LocalComm()
        self.stream = stream
        self._heavy_pre = None          # id(col) -> heavy keys sampled with pass 1
        self._near_unique = set()       # id(col) of columns >= 90 % distinct in that sample
        self._counted = {}              # id(col) -> group context whose level-1 count pass 2 did
        self._heavy_bytes_pre = {}      # id(col) -> byte column's heavy keys, sampled with pass 1

    # -- small helpers ----------------------------------------------------------

    def _s(self):
        return nat.stream_handle(self.stream)

    def _bytes(self, n):
        return torch.empty(max(int(n), 16), dtype=torch.uint8, device=self.device)

    def _u64(self, n, zero=False):
        f = torch.zeros if zero else torch.empty
        return f(max(int(n), 1), dtype=torch.int64, device=self.device)

    @staticmethod
    def _read(t, cls):
        b = t[:ctypes.sizeof(cls)].cpu().numpy().tobytes()
        return cls.from_buffer_copy(b)

    def _to_dev(self, struct):
        # (through _h2d: on self.stream, ahead of the kernels that read the
        # table there; comm.to_dev stays for tensors torch ops consume on the
        # current stream)
        return self._h2d(np.frombuffer(bytearray(bytes(struct)), dtype=np.uint8))


    def _h2d(self, arr):
        """Host numpy array -> device tensor without a host round trip: staged
        through pinned memory and copied asynchronously on the engine's stream
        (a pageable copy would wait for every kernel queued before it)."""
        t = torch.from_numpy(np.ascontiguousarray(arr))
        with torch.cuda.stream(self.stream) if self.stream is not None else _nullctx():
            return t.pin_memory().to(self.device, non_blocking=True)

    @staticmethod
    def _host_u64(t):
        return [int(x) & U64 for x in t.cpu().numpy().view(np.uint64).tolist()]

    # ==========================================================================
    # numeric columns
    # ==========================================================================
    def plan(self, col: DeviceColumn, probs=PROBS):
        world = self.comm.world
        ns = max(1, SAMPLE_TOTAL // world)
        sample = self._u64(ns)
        cs = col.sdp()
        sdp.sdp_sample_keys(ctypes.byref(cs), ns, ptr(sample), self._s())
        parts = self.comm.allgather(sample)
        allk = torch.cat(parts) if len(parts) > 1 else sample
        pr = self._h2d(np.array(list(probs), dtype=np.float64))
        plan_dev = self._bytes(ctypes.sizeof(nat.SdpQPlan))
        sdp.sdp_quantile_plan(ptr(allk), allk.numel(), ptr(pr), len(probs), int(col.is_float), ptr(plan_dev),
                              self._s())
        return plan_dev, self._read(plan_dev, nat.SdpQPlan)

    def empty_plan(self):
        p = nat.SdpQPlan()
        p.n_windows = 0
        p.shift = 0.0
        return self._to_dev(p), p

    def _pass1_launch(self, col: DeviceColumn, plan_dev, plan, res_dev=None, budget=None, defer=False):
        """Launch pass 1 of one column.  `budget` (a one-element list of bytes
        left) is shared by the columns of one batch: every column's candidate
        slots stay alive until its quantiles are resolved, so the room-for-
        every-row sizing below is granted only while the batch's total stays
        under CAND_FULL_BUDGET; past it (wide tables: 512 columns x 1e7 rows
        would need ~350 GB) slots are sized from the sample estimate, whose
        rare overflow falls back to the exact whole-column select."""
        n = col.length
        grid = sdp.sdp_pass1_grid(n, col.dtype)
        work = self._bytes(sdp.sdp_pass1_workspace_bytes(n, col.dtype))
        nw = plan.n_windows
        nseg = grid * nat.PASS1_WAVES                    # wave-private candidate segments per window
        cap = 0
        if nw:
            rows_pb = n / max(grid, 1)
            for w in range(nw):
                frac = 1.0 if plan.n_sample < 64 else min(1.0, (plan.in_sample[w] + 2.0) / plan.n_sample)
                exp = frac * rows_pb
                cap = max(cap, int(2.0 * exp + 6.0 * math.sqrt(exp) + 64))
            # a block's rows come from whole grid-strided tiles; at small n a window
            # can sit inside one tile (sorted data), so give every block room for
            # all its rows when the batch can afford it
            tile_rows = 256 * 4 * (16 // nat.ELEM_SIZE[col.dtype])
            full = int(math.ceil(n / max(grid, 1) / tile_rows + 1)) * tile_rows
            full_bytes = nw * nseg * (-(-full // nat.PASS1_WAVES) + 64) * 8
            if budget is None:
                budget = [CAND_FULL_BUDGET]
            if n <= (1 << 24) and full_bytes <= budget[0]:
                cap = full
                budget[0] -= full_bytes
            else:
                cap = min(cap, full)
        cap = -(-cap // nat.PASS1_WAVES) + 64 if cap else 0
        if nw and DEBUG_QUANTILE == 'overflow':
            cap = 1                                       # every busy segment overflows
        cand = self._u64(max(nw, 1) * nseg * max(cap, 1))
        cand_counts = torch.zeros(max(nw, 1) * nseg, dtype=torch.int32, device=self.device)
        if res_dev is None:
            res_dev = self._bytes(ctypes.sizeof(nat.SdpPass1Result))
        cs = col.sdp()
        # inclusive windows when no used window needs exclusive bounds (see sdp_qplan.excl_mask)
        flags = 1 if (nw and PASS1_INCLUSIVE and not (plan.excl_mask & ((1 << nw) - 1))) else 0
        info = {'cand': cand, 'counts': cand_counts, 'nseg': nseg, 'cap': cap, 'res_dev': res_dev}
        if defer:
            # sdp_pass1_batch task: launched with the other columns of its kind
            info['task'] = nat.SdpPass1Task(cs, plan_dev.data_ptr(), work.data_ptr(), cand.data_ptr(),
                                            cand_counts.data_ptr(), cap, res_dev.data_ptr(), grid, 0)
            info['kind'] = (col.dtype, int(cap > 0), flags)
            info['work'] = work
            info['col'] = col
            return info
        nat.annotate(_label(col), col_read_bytes(col))
        sdp.sdp_pass1(ctypes.byref(cs), ptr(plan_dev), ptr(work), work.numel(), ptr(cand), ptr(cand_counts), cap,
                      flags, ptr(res_dev), self._s())
        return info

    def _pass1_run_batch(self, infos):
        """Launch deferred pass-1 tasks (_pass1_launch(defer=True)): one
        sdp_pass1_batch per (dtype, windowed, flags) kind; a kind with one
        column takes the single-column entry."""
        kinds = {}
        for inf in infos:
            kinds.setdefault(inf['kind'], []).append(inf)
        keep = []
        for (dtype, windowed, flags), grp in kinds.items():
            if len(grp) == 1:
                inf = grp[0]
                t = inf['task']
                nat.annotate(_label(inf['col']), col_read_bytes(inf['col']))
                sdp.sdp_pass1(ctypes.byref(t.col), ctypes.c_void_p(t.d_plan), ctypes.c_void_p(t.d_work),
                              inf['work'].numel(), ctypes.c_void_p(t.d_cand), ctypes.c_void_p(t.d_cand_counts),
                              t.slot_capacity, flags, ctypes.c_void_p(t.d_result), self._s())
                continue
            arr = (nat.SdpPass1Task * len(grp))(*[inf['task'] for inf in grp])
            d_tasks = self._h2d(np.frombuffer(bytearray(bytes(arr)), dtype=np.uint8))
            nat.annotate(_label(grp[0]['col'], 'batch'), sum(col_read_bytes(inf['col']) for inf in grp))
            sdp.sdp_pass1_batch(ptr(d_tasks), len(grp), dtype, windowed, flags, max(inf['task'].grid for inf in grp),
                                self._s())
            keep.append(d_tasks)
        for inf in infos:
            for k in ('task', 'kind', 'work', 'col'):
                inf.pop(k, None)
        return keep

    def pass1(self, col: DeviceColumn, plan_dev, plan):
        info = self._pass1_launch(col, plan_dev, plan)
        local = self._read(info['res_dev'], nat.SdpPass1Result)
        return local, info

    def merge_pass1(self, local: nat.SdpPass1Result):
        """All-gather the per-rank pass-1 states and merge them in rank order."""
        if not self.comm.sharded:
            return merge_pass1_results([local])
        raw = to_dev(np.frombuffer(bytearray(bytes(local)), dtype=np.uint8), torch.uint8, self.device)
        parts = [nat.SdpPass1Result.from_buffer_copy(p.cpu().numpy().tobytes()) for p in self.comm.allgather(raw)]
        return merge_pass1_results(parts)

    def select_kth(self, keys, n_dev, k, lo_key, hi_key):
        """k-th smallest (0-based) key over every rank's `keys[:n]`; all keys lie
        in [lo_key, hi_key].  Radix rounds of 11 bits with all-reduced digit
        histograms; the final bucket (<= SORT_MAX keys) is gathered and sorted."""
        comm = self.comm
        total = int(comm.allreduce_sum(n_dev.clone()).item())
        if k < 0 or k >= total:
            raise RuntimeError('select_kth: rank %d outside %d keys' % (k, total))
        x = _u(lo_key) ^ _u(hi_key)
        shift = ((x.bit_length() - 1) // 11) * 11 if x else 0
        prefix = (_u(lo_key) >> (shift + 11)) if shift + 11 < 64 else 0
        cur, cur_n = keys, n_dev
        while True:
            if total <= SORT_MAX:
                return self._gather_sorted_pick(cur, cur_n, k)
            hist = self._u64(2048, zero=True)
            sdp.sdp_radix_hist(ptr(cur), ptr(cur_n), prefix, shift, ptr(hist), self._s())
            hist = comm.allreduce_sum(hist)
            h = hist.cpu().numpy().view(np.uint64).astype(np.int64)
            cum = np.cumsum(h)
            j = int(np.searchsorted(cum, k, side='right'))
            before = int(cum[j - 1]) if j > 0 else 0
            k -= before
            total = int(h[j])
            prefix = ((prefix << 11) | j) & U64
            if shift == 0:
                return prefix
            nxt = self._u64(max(int(cur.numel()), 1))
            nxt_n = self._u64(1, zero=True)
            sdp.sdp_radix_filter(ptr(cur), ptr(cur_n), prefix, shift, ptr(nxt), ptr(nxt_n), self._s())
            cur, cur_n = nxt, nxt_n
            shift -= 11

    def _gather_sorted_pick(self, cur, cur_n, k):
        n_local = int(cur_n.item())
        mine = cur[:n_local]
        parts = self.comm.allgatherv(mine)
        allk = torch.cat(parts) if len(parts) > 1 else mine.clone()
        nn = torch.full((1,), allk.numel(), dtype=torch.int64, device=self.device)
        buf = self._u64(max(allk.numel(), 1))
        buf[:allk.numel()] = allk
        sdp.sdp_sort_small(ptr(buf), ptr(nn), self._s())
        return _u(buf[k].item())

    def resolve_quantiles(self, col, p1: dict, plan, cand_info, probs=PROBS):
        """Order statistics for each requested probability (describe.py:203-208)."""
        return self.quantiles_batch([(col, p1, plan, cand_info)], probs)[0]

    @staticmethod
    def _rank_key_range(r, p1, plan):
        """The key range [a, b] (inclusive) and rank span [base, base + cnt) of
        the na.drop keys that rank r (0-based) falls among when no window
        resolves it: the gap between two pass-1 windows (or before the first /
        after the last), or an overflowed window itself.  Exact from pass 1's
        merged counts, identical on every rank."""
        n = p1['count']
        a, start = 0, 0
        for w in range(plan.n_windows):
            size = p1['w_eq_lo'][w] + p1['w_in'][w] + p1['w_eq_hi'][w]
            below = n - p1['w_gt'][w] - size
            if r < below:
                return a, _u(plan.lo[w]) - 1, start, below - start
            if r < below + size:
                return _u(plan.lo[w]), _u(plan.hi[w]), below, size
            a, start = _u(plan.hi[w]) + 1, below + size
        return a, EMPTY64, start, n - start

    def _range_keys(self, col, a, b, cap):
        """The na.drop keys of `col` in [a, b] (at most `cap` of them locally)."""
        out = self._u64(max(int(cap), 1))
        out_n = self._u64(1, zero=True)
        cs = col.sdp()
        nat.annotate(_label(col, 'range_keys'), col_read_bytes(col))
        sdp.sdp_column_keys_range(ctypes.byref(cs), _u(a), _u(b), ptr(out), ptr(out_n), self._s())
        return out, out_n

    def pass2(self, col, mean, edges, hi_t, lo_t):
        bins = len(edges)
        e = self._h2d(np.array([float(x) for x in edges], dtype=np.float64))
        mono = all(math.isfinite(float(x)) for x in edges) and all(
            float(edges[i]) <= float(edges[i + 1]) for i in range(bins - 1))
        need = sdp.sdp_pass2_workspace_bytes(col.length, col.dtype, bins)
        work = self._bytes(need)
        res = self._bytes(ctypes.sizeof(nat.SdpPass2Result))
        hist = self._u64(bins)
        cs = col.sdp()
        nat.annotate(_label(col), col_read_bytes(col))
        sdp.sdp_pass2(ctypes.byref(cs), float(mean), ptr(e), bins, int(mono), float(hi_t), float(lo_t), ptr(work),
                      work.numel(), ptr(res), ptr(hist), self._s())
        if not self.comm.sharded:        # result struct and bins in one readback
            sz = ctypes.sizeof(nat.SdpPass2Result)
            raw = torch.cat([res[:sz], hist.view(torch.uint8)]).cpu().numpy()
            r = nat.SdpPass2Result.from_buffer_copy(raw[:sz].tobytes())
            return {'abs_dev_sum': float(r.abs_dev_sum), 'n_high': int(r.n_high), 'n_low': int(r.n_low),
                    'n_unbinned': int(r.n_unbinned), 'hist': raw[sz:].view(np.int64).astype(np.int64)}
        r = self._read(res, nat.SdpPass2Result)
        # merge ranks: counts sum exactly; abs-dev sums gathered and added in rank order
        vec = to_dev([r.n_high, r.n_low, r.n_unbinned], torch.int64, self.device)
        vec = self.comm.allreduce_sum(torch.cat([vec, hist]))
        mads = self.comm.allgather(torch.full((1,), r.abs_dev_sum, dtype=torch.float64, device=self.device))
        v = vec.cpu().numpy()
        return {'abs_dev_sum': math.fsum(float(m.item()) for m in mads), 'n_high': int(v[0]), 'n_low': int(v[1]),
                'n_unbinned': int(v[2]), 'hist': v[3:].astype(np.int64)}

    def numeric_stats(self, col, bins=10, k=2, probs=PROBS, p1_pack=None):
        """Everything describe_numeric_1d computes except the PNG strings."""
        if p1_pack is None:
            p1_pack = self.numeric_pass1(col, probs)
        p1, plan, cand_info = p1_pack
        n = p1['count']
        is_int = not col.is_float
        mom = moments(p1, is_int)
        qs, fb = self.resolve_quantiles(col, p1, plan, cand_info, probs)
        st = NumericStats(count=n, n_valid=p1['n_valid'], n_nan=p1['n_nan'], n_zero=p1['n_zero'], **mom)
        st.quantiles = qs
        st.fallback_used = fb
        q1, q3 = qs[0.25], qs[0.75]
        hi_t = q3 + k * (q3 - q1)                          # describe.py:222
        lo_t = q1 - k * (q3 - q1)                          # describe.py:223
        edges, width = hist_edges(st.min, st.max, bins)   # describe.py:226 -> :40-45
        r2 = self.pass2(col, st.mean, edges, hi_t, lo_t)
        st.mad = r2['abs_dev_sum']
        st.hist_counts = r2['hist']
        st.edges = edges
        st.width = width
        st.high_idx = r2['n_high']
        st.low_idx = r2['n_low']
        st.thresholds = (hi_t, lo_t)
        return st

    # ==========================================================================
    # whole-table batches: every numeric column's order statistics, then every
    # column's pass 2, each with ONE host readback (one collective set when
    # sharded) instead of one or more per column
    # ==========================================================================
    def _queue_column_selects(self, ci, col, p1, plan, cand_info, probs, dense_req, selects, fallbacks):
        """Decide, for each rank a column needs (describe.py:203-208), whether a
        window bound resolves it from pass-1's counts or a select must run in a
        window's compacted candidates (the window is appended to `dense_req` as
        (column, window, dense capacity, cand_info) and the select to `selects`
        as [rank, ('dense', request), None, cap, k, lo, hi, cap]).  A rank no
        window resolves (missed window, overflowed slots) goes to `fallbacks`
        as (rank, key range [a, b], first rank of the range, keys in it).  The
        returned state is finished by _finish_column_quantiles."""
        n = p1['count']
        is_int = not col.is_float
        needed = {}
        for p in probs:
            if is_int:
                pos = (n - 1) * p
                needed[p] = (pos, math.floor(pos), math.ceil(pos))
            else:
                needed[p] = (None, spark_percentile_approx_rank(n, p) - 1, None)
        ranks = sorted({r for v in needed.values() for r in (v[1], v[2]) if r is not None})
        values, dense = {}, {}
        w_eq_lo, w_in, w_gt, w_eq_hi = p1['w_eq_lo'], p1['w_in'], p1['w_gt'], p1['w_eq_hi']
        for r in ranks:
            key = None
            for w in range(plan.n_windows):
                size = w_eq_lo[w] + w_in[w] + w_eq_hi[w]
                below = n - w_gt[w] - size
                if below <= r < below + size:
                    rr = r - below
                    lo, hi = plan.lo[w], plan.hi[w]
                    if rr < w_eq_lo[w]:
                        key = lo
                    elif rr < w_eq_lo[w] + w_in[w]:
                        if (p1['w_overflow'] >> w) & 1:
                            break
                        if w not in dense:
                            # dense copy sized by the window's (global) inside count
                            dense[w] = len(dense_req)
                            dense_req.append((ci, w, max(1, int(w_in[w])), cand_info))
                        cap = dense_req[dense[w]][2]
                        selects.append([r, ('dense', dense[w]), None, cap, rr - w_eq_lo[w], lo, hi, cap])
                        key = 'queued'
                    else:
                        key = hi
                    break
            if key is None:
                fallbacks.append((r,) + self._rank_key_range(r, p1, plan))
                key = 'queued'
            values[r] = key
        return {'values': values, 'needed': needed, 'is_int': is_int, 'probs': probs, 'fallback': False}

    SELECT_BATCH_BYTES = 24 << 30          # select workspaces alive at once (flushed in groups)
    BYTES_BATCH_BYTES = 40 << 30           # byte columns' (key, count) group outputs alive at once
    _sel_ws0 = None

    @classmethod
    def _select_ws(cls, n_cap):
        """sdp_select_kth_workspace_bytes(n_cap) (sdp_numeric.hip: 256-byte
        aligned state, histogram, two counters, two key buffers) without a
        foreign call per select."""
        if cls._sel_ws0 is None:
            cls._sel_ws0 = int(sdp.sdp_select_kth_workspace_bytes(1)) - 512
        return cls._sel_ws0 + 2 * ((8 * max(int(n_cap), 1) + 255) // 256 * 256)

    @staticmethod
    def _select_rounds(lo, hi):
        x = _u(lo) ^ _u(hi)
        return (x.bit_length() - 1) // 11 + 1 if x else 1      # sdp_select_rounds

    def _run_selects(self, selects, res):
        """Queue every select of `selects` ([rank, keys pointer, count pointer,
        n_cap, k, lo, hi, budget_cap]); result j lands in res[j].  Groups whose
        workspaces fit SELECT_BATCH_BYTES run as one sdp_select_batch (sharded:
        one stream-ordered all-reduce of the digit histograms per radix round
        for the whole group).  Returns the buffers that must outlive the
        readback."""
        s = self._s()
        keep = []
        j0 = 0
        ws = [self._select_ws(x[7]) for x in selects]
        wsa = [(w + 255) // 256 * 256 for w in ws]
        while j0 < len(selects):
            # a group of selects whose workspaces fit the budget (at least one);
            # budget_cap is the same on every rank, so is the grouping
            j1, tot = j0, 0
            while j1 < len(selects):
                if j1 > j0 and tot + ws[j1] > self.SELECT_BATCH_BYTES:
                    break
                tot += wsa[j1]
                j1 += 1
            q = j1 - j0
            sizes = [self._select_ws(x[3]) for x in selects[j0:j1]]
            offs = np.concatenate([[0], np.cumsum([(w + 255) // 256 * 256 for w in sizes])]).astype(np.uint64)
            work = self._bytes(int(offs[-1]))
            t = np.zeros((q, 8), dtype=np.uint64)           # SdpSelectTask rows
            grp = selects[j0:j1]
            t[:, 0] = [x[1] for x in grp]
            t[:, 1] = [x[2] for x in grp]
            t[:, 2] = [int(x[3]) for x in grp]
            t[:, 3] = [int(x[4]) for x in grp]
            t[:, 4] = [_u(x[5]) for x in grp]
            t[:, 5] = [_u(x[6]) for x in grp]
            t[:, 6] = np.uint64(work.data_ptr()) + offs[:-1]
            t[:, 7] = np.uint64(res.data_ptr()) + np.uint64(8) * np.arange(j0, j1, dtype=np.uint64)
            rounds = max(self._select_rounds(x[5], x[6]) for x in grp)
            d_tasks = self._h2d(t.view(np.uint8).reshape(-1))
            hist = self._u64(q * 2048)
            if not self.comm.sharded:
                sdp.sdp_select_batch(ptr(d_tasks), q, rounds, ptr(hist), s)
            else:
                sdp.sdp_select_batch_init(ptr(d_tasks), q, ptr(hist), s)
                for rd in range(rounds):
                    self.comm.allreduce_sum_(hist)
                    sdp.sdp_select_batch_step(ptr(d_tasks), q, rd, int(rd == rounds - 1), ptr(hist), s)
            keep.append((d_tasks, work, hist))
            j0 = j1
        return keep

    def quantiles_batch(self, items, probs=PROBS):
        """[(col, p1, plan, cand_info)] -> [(quantiles, fallback_used)] with
        the candidate compactions of every window in two launches, the selects
        of every column in ~2 launches per radix round (sdp_select_batch; one
        all-reduce per round for ALL columns when sharded) and one readback.
        The dense candidate copies of all windows share one allocation and
        every task table is built as one numpy array (wide tables: 512 columns
        x 5 windows).  Ranks no window resolves are then selected one key
        range at a time: the range's keys are re-collected from the column
        (sized by pass 1's exact count), selected and freed, so the fallback
        holds at most one range (<= 24 B per row of it) instead of every
        column's keys."""
        s = self._s()
        states, sel_owner, dense_req, selects, fbs = [], [], [], [], []
        for i, (col, p1, plan, cand_info) in enumerate(items):
            before = len(selects)
            fb = []
            states.append(self._queue_column_selects(i, col, p1, plan, cand_info, probs, dense_req, selects, fb))
            sel_owner += [i] * (len(selects) - before)
            fbs.append(fb)
        keep = []
        if dense_req:
            m = len(dense_req)
            caps = np.array([d[2] for d in dense_req], dtype=np.uint64)
            coff = np.concatenate([[0], np.cumsum(caps)]).astype(np.uint64)
            nsegs = np.array([d[3]['nseg'] for d in dense_req], dtype=np.uint64)
            noff = np.concatenate([[0], np.cumsum(nsegs)]).astype(np.uint64)
            dbuf = self._u64(int(coff[-1]))
            dn = self._u64(m, zero=True)
            offw = self._u64(int(noff[-1]))
            t = np.zeros((m, 7), dtype=np.uint64)           # SdpCompactTask rows
            t[:, 0] = [d[3]['cand'].data_ptr() + 8 * d[1] * d[3]['nseg'] * d[3]['cap'] for d in dense_req]
            t[:, 1] = [d[3]['counts'].data_ptr() + 4 * d[1] * d[3]['nseg'] for d in dense_req]
            t[:, 2] = nsegs
            t[:, 3] = [d[3]['cap'] for d in dense_req]
            t[:, 4] = np.uint64(offw.data_ptr()) + np.uint64(8) * noff[:-1]
            t[:, 5] = np.uint64(dbuf.data_ptr()) + np.uint64(8) * coff[:-1]
            t[:, 6] = np.uint64(dn.data_ptr()) + np.uint64(8) * np.arange(m, dtype=np.uint64)
            d_tasks = self._h2d(t.view(np.uint8).reshape(-1))
            sdp.sdp_compact_batch(ptr(d_tasks), m, int(nsegs.max()), s)
            keep.append((d_tasks, dbuf, dn, offw))
            for x in selects:                                 # ('dense', j) -> the j-th dense copy
                j = x[1][1]
                x[1] = dbuf.data_ptr() + 8 * int(coff[j])
                x[2] = dn.data_ptr() + 8 * j
        res = self._u64(max(1, len(selects)))
        keep += self._run_selects(selects, res)
        keys = self._host_u64(res) if selects else []          # the one readback
        del keep
        for j, owner in enumerate(sel_owner):
            states[owner]['values'][selects[j][0]] = keys[j]
        del selects
        # fallback ranks, one key range at a time (the same sequence on every rank)
        for i, (col, p1, plan, cand_info) in enumerate(items):
            groups = {}
            for r, a, b, base, cnt in fbs[i]:
                groups.setdefault((a, b, base, cnt), []).append(r)
            for (a, b, base, cnt), rs in groups.items():
                arr, arr_n = self._range_keys(col, a, b, min(int(cnt), col.length))
                sel = [[r, arr.data_ptr(), arr_n.data_ptr(), arr.numel(), r - base, a, b, max(1, int(cnt))]
                       for r in rs]
                res = self._u64(len(sel))
                keep = self._run_selects(sel, res)
                for r, v in zip(rs, self._host_u64(res)):
                    states[i]['values'][r] = v
                del keep, arr, arr_n, sel
                states[i]['fallback'] = True
        return [self._finish_column_quantiles(st) for st in states]

    @staticmethod
    def _finish_column_quantiles(st):
        values, needed, is_int = st['values'], st['needed'], st['is_int']
        out = {}
        for p in st['probs']:
            pos, lo_r, hi_r = needed[p]
            if is_int:
                lk, hk = key_to_int(values[lo_r]), key_to_int(values[hi_r])
                if hi_r == lo_r or hk == lk:
                    out[p] = float(lk)
                else:       # Spark Percentile linear interpolation (A.4)
                    out[p] = (hi_r - pos) * float(lk) + (pos - lo_r) * float(hk)
            else:
                out[p] = key_to_float(values[lo_r])
        return out, st['fallback']

    def pass2_batch(self, items, count_ctx=None):
        """[(col, mean, edges, hi_t, lo_t)] -> [pass-2 dict] (see pass2), all
        launched back to back and read back once (sharded: one all-reduce of
        every column's counts and bins, one all-gather of the mad partials).
        count_ctx[i] (a _group_prepare context) makes column i's launch also do
        the level-1 count of its distinct-count partitioning (sdp_pass2_count);
        the context is then kept for group_batch."""
        if not items:
            return []
        count_ctx = count_ctx or {}
        s = self._s()
        rsz = ctypes.sizeof(nat.SdpPass2Result)
        outs = []
        batched = []               # (kind, SdpPass2Task, col): counted columns launched together below
        for i, (col, mean, edges, hi_t, lo_t) in enumerate(items):
            bins = len(edges)
            e = self._h2d(np.array([float(x) for x in edges], dtype=np.float64))
            mono = all(math.isfinite(float(x)) for x in edges) and all(
                float(edges[j]) <= float(edges[j + 1]) for j in range(bins - 1))
            res = self._bytes(rsz)
            hist = self._u64(bins)
            cs = col.sdp()
            ctx = count_ctx.get(i)
            batch = PASS2_BATCH and len(items) >= 8
            if ctx is not None and ctx.get('d32') and not batch:
                ctx = None                  # (the d32 pre-count rides the batched launch only)
            if ctx is not None:
                work = self._bytes(max(sdp.sdp_pass2_count_workspace_bytes(col.length, bins),
                                       sdp.sdp_pass2_workspace_bytes(col.length, col.dtype, bins)))
                hv = ctx['hv']
                if batch:
                    rpb = sdp.sdp_part_rows_per_block(col.length, 0)
                    grid = max(1, -(-col.length // rpb))
                    task = nat.SdpPass2Task(cs, e.data_ptr(), float(mean), float(hi_t), float(lo_t), work.data_ptr(),
                                            res.data_ptr(), hist.data_ptr(),
                                            hv['struct'] if hv else nat.SdpHeavy(None, None, None, None, 0, 0),
                                            ctx['h1'].data_ptr(), ctx['hcnt'].data_ptr(), ctx['stats'].data_ptr(),
                                            rpb, bins, int(mono), ctx['b1'], grid, int(ctx.get('lo', 0)))
                    batched.append(((col.dtype, bins, int(mono)), task, col))
                else:
                    nat.annotate(_label(col), col_read_bytes(col))
                    sdp.sdp_pass2_count(ctypes.byref(cs), float(mean), ptr(e), bins, int(mono), float(hi_t),
                                        float(lo_t), ptr(work), work.numel(), ptr(res), ptr(hist),
                                        ctypes.byref(hv['struct']) if hv else None, ctx['b1'], ptr(ctx['h1']),
                                        ptr(ctx['hcnt']), ptr(ctx['stats']), s)
                self._counted[id(col)] = ctx
            else:
                work = self._bytes(sdp.sdp_pass2_workspace_bytes(col.length, col.dtype, bins))
                nat.annotate(_label(col), col_read_bytes(col))
                sdp.sdp_pass2(ctypes.byref(cs), float(mean), ptr(e), bins, int(mono), float(hi_t), float(lo_t),
                              ptr(work), work.numel(), ptr(res), ptr(hist), s)
            outs.append((res, hist, e, work))
        keep_tasks = []
        if batched:
            # wide tables: one sdp_pass2_count_batch per (dtype, bins, edge kind)
            kinds = {}
            for kind, task, col in batched:
                kinds.setdefault(kind, []).append((task, col))
            for (dtype, bins, mono), grp in kinds.items():
                mg = max(t.grid for t, _ in grp)
                for t, c in grp:      # sdp_pass2_count's own argument checks (the table is device memory)
                    if (c.values.data_ptr() % 16 or not -1 <= t.b1 <= 10 or t.heavy.n > nat.HEAVY_MAX
                            or (t.b1 == -1 and c.dtype not in (nat.F32,) + self.BITS32_DTYPES)
                            or t.grid > mg or mg > nat.PART_MAX_GRID):
                        raise nat.NativeError('pass2_count_batch: a task fails the sdp_pass2_count checks')
                arr = (nat.SdpPass2Task * len(grp))(*[t for t, _ in grp])
                d_tasks = self._h2d(np.frombuffer(bytearray(bytes(arr)), dtype=np.uint8))
                nat.annotate(_label(grp[0][1], 'batch'), sum(col_read_bytes(c) for _, c in grp))
                sdp.sdp_pass2_count_batch(ptr(d_tasks), len(grp), dtype, bins, mono, mg, s)
                keep_tasks.append(d_tasks)
        return self._pass2_results(outs)

    def _pass2_results(self, outs):
        """The pass-2 dicts of launched columns [(res, hist, edges, work)]: one
        readback (sharded: one all-gather)."""
        rsz = ctypes.sizeof(nat.SdpPass2Result)
        if not self.comm.sharded:
            raw = torch.cat([t for res, hist, _, _ in outs for t in (res[:rsz], hist.view(torch.uint8))]).cpu().numpy()
            result, off = [], 0
            for (res, hist, _, _) in outs:
                r = nat.SdpPass2Result.from_buffer_copy(raw[off:off + rsz].tobytes())
                off += rsz
                hb = hist.numel() * 8
                result.append({'abs_dev_sum': float(r.abs_dev_sum), 'n_high': int(r.n_high), 'n_low': int(r.n_low),
                               'n_unbinned': int(r.n_unbinned),
                               'hist': raw[off:off + hb].view(np.int64).astype(np.int64)})
                off += hb
            return result
        # sharded: counts and bins summed exactly; abs-dev partials gathered, summed in rank order
        # (one all-gather and one readback: the int64 counts are summed over
        # ranks on the host, exactly, the fp64 partials in rank order)
        parts = torch.cat([torch.cat([res[:rsz].view(torch.int64)[1:4], hist]) for res, hist, _, _ in outs])
        mads = torch.stack([res[:8].view(torch.float64)[0] for res, _, _, _ in outs])
        allp = torch.stack(self.comm.allgather(torch.cat([parts, mads.view(torch.int64)]))).cpu().numpy()
        summed = allp[:, :parts.numel()].sum(axis=0)
        allm = np.ascontiguousarray(allp[:, parts.numel():]).view(np.float64)   # [world, ncols]
        result, off = [], 0
        for i, (res, hist, _, _) in enumerate(outs):
            v = summed[off:off + 3 + hist.numel()]
            off += 3 + hist.numel()
            result.append({'abs_dev_sum': math.fsum(float(x) for x in allm[:, i]), 'n_high': int(v[0]),
                           'n_low': int(v[1]), 'n_unbinned': int(v[2]), 'hist': v[3:].astype(np.int64)})
        return result

    def gk_quantiles(self, col: DeviceColumn, probs=PROBS, partitions=1, accuracy=10000):
        """percentile_approx(c, p, accuracy) (describe.py:205-206) as Spark 2.x's
        ApproximatePercentile returns it when the column's rows form `partitions`
        contiguous Spark partitions merged in partition order (sdp_gk_quantiles;
        oracle/gk.py restates the algorithm).  On a row-sharded table rank r's
        rows form partitions r*k .. r*k+k-1 (k = partitions / world) and the
        digests are merged across ranks in partition order."""
        return self.gk_quantiles_batch([col], probs, partitions, accuracy)[0]

    def gk_quantiles_batch(self, cols, probs=PROBS, partitions=1, accuracy=10000):
        """gk_quantiles of several columns: single rank, every column's GK
        kernels queued back to back and ONE readback of all statuses and
        results.  The GK build runs one workgroup per Spark partition with a
        sequential compress scan, so few partitions over many rows leave the
        GPU mostly idle (a correctness mode: see DESIGN.md)."""
        partitions = int(partitions)
        if self.comm.sharded:
            return [self._gk_quantiles_sharded(c, probs, partitions, accuracy) for c in cols]
        if partitions < 64 and any(c.length > 10 ** 7 for c in cols):
            import warnings
            warnings.warn('quantile_mode="gk" with %d Spark partition(s) over %d rows: the GK build is one '
                          'workgroup per partition; expect seconds per column (spark_partitions sets P)'
                          % (partitions, max(c.length for c in cols)), RuntimeWarning, stacklevel=3)
        wb = sdp.sdp_gk_workspace_bytes(partitions)
        pr = self._h2d(np.asarray(probs, dtype=np.float64))
        npb = max(len(probs), 1)
        out = torch.empty(len(cols) * npb, dtype=torch.float64, device=self.device)
        status = self._u64(3 * len(cols), zero=True)
        work = self._bytes(wb)                 # reused: launches on one stream run in order
        for i, col in enumerate(cols):
            cs = col.sdp()
            nat.annotate('gk', col_read_bytes(col))
            sdp.sdp_gk_quantiles(ctypes.byref(cs), partitions, int(accuracy), ptr(pr), len(probs), ptr(work), wb,
                                 ptr(out[i * npb:]), ptr(status[3 * i:]), self._s())
        host = torch.cat([status.view(torch.float64), out]).cpu().numpy()
        st = host[:3 * len(cols)].view(np.int64)
        vals = host[3 * len(cols):]
        res = []
        for i in range(len(cols)):
            if st[3 * i]:
                raise RuntimeError('sdp_gk_quantiles: summary capacity exceeded (status %d)' % int(st[3 * i]))
            res.append({p: float(v) for p, v in zip(probs, vals[i * npb:(i + 1) * npb])})
        return res

    def _gk_quantiles_sharded(self, col, probs, partitions, accuracy):
        """gk_quantiles of a row-sharded column: rank r's rows form Spark
        partitions r*k .. r*k + k - 1 (k = partitions / world, each a
        contiguous share of the rank's rows); every rank builds its own
        partition digests, the digests are all-gathered, and every rank merges
        all of them in partition order (identical results everywhere)."""
        comm, world = self.comm, self.comm.world
        if partitions % world:
            raise ValueError('spark_partitions must be a multiple of the number of ranks')
        k = partitions // world

        def layout(P):
            lay = (ctypes.c_int64 * 4)()
            sdp.sdp_gk_layout(P, ctypes.addressof(lay))
            return [int(x) for x in lay]

        s = self._s()
        head, pb, boff, cap = layout(k)
        wb = sdp.sdp_gk_workspace_bytes(k)
        work = self._bytes(wb)
        cs = col.sdp()
        nat.annotate('gk', col_read_bytes(col))
        sdp.sdp_gk_partitions(ctypes.byref(cs), k, int(accuracy), ptr(work), wb, s)
        states = work[:k * 32].view(torch.int64).view(k, 4)
        st = states.cpu().numpy()
        pieces = [states.reshape(-1)]
        for j in range(k):
            n_j, which = int(st[j, 0]), int(st[j, 2])
            base = head + j * pb + boff + which * cap * 24
            for f in range(3):                       # v (f64 bits), g, d
                pieces.append(work[base + f * cap * 8: base + f * cap * 8 + n_j * 8].view(torch.int64))
        parts = comm.allgatherv(torch.cat(pieces))
        head2, pb2, boff2, cap2 = layout(partitions)
        wb2 = sdp.sdp_gk_workspace_bytes(partitions)
        work2 = torch.zeros(wb2, dtype=torch.uint8, device=self.device)
        hdr = torch.zeros((partitions, 4), dtype=torch.int64, device=self.device)
        for r, pk in enumerate(parts):
            sth = pk[:k * 4].view(k, 4).cpu().numpy()
            off = k * 4
            for j in range(k):
                p, n_j = r * k + j, int(sth[j, 0])
                hdr[p, 0], hdr[p, 1], hdr[p, 2], hdr[p, 3] = n_j, int(sth[j, 1]), 0, int(sth[j, 3])
                base = head2 + p * pb2 + boff2
                for f in range(3):
                    work2[base + f * cap2 * 8: base + f * cap2 * 8 + n_j * 8].view(torch.int64)[:] = pk[off:off + n_j]
                    off += n_j
        work2[:partitions * 32].view(torch.int64)[:] = hdr.reshape(-1)
        pr = self._h2d(np.asarray(probs, dtype=np.float64))
        out = torch.empty(max(len(probs), 1), dtype=torch.float64, device=self.device)
        status = self._u64(3, zero=True)
        sdp.sdp_gk_merge(partitions, int(accuracy), ptr(pr), len(probs), ptr(work2), wb2, ptr(out), ptr(status), s)
        stv = status.cpu().numpy()
        if stv[0]:
            raise RuntimeError('sdp_gk_merge: summary capacity exceeded (status %d)' % int(stv[0]))
        return {p: float(v) for p, v in zip(probs, out.cpu().numpy())}

    def numeric_stats_batch(self, cols, packs, bins=10, ks=None, probs=PROBS, group_cols=(), gk=None,
                            count32_cols=None):
        """numeric_stats of every column (None for a column with no non-null
        value) with two host readbacks in all.  A bins value the reference
        rejects (describe.py:46 with bins=1) is recorded per column and raised
        when describe_1d reaches that column, as the reference would."""
        ks = ks or [2] * len(cols)
        live = [i for i, pk in enumerate(packs) if pk[0]['count'] > 0]
        # quantile_mode='gk': float columns take Spark's percentile_approx
        # element (also the q1/q3 of the outlier thresholds, as
        # describe.py:212-223 uses them) and skip the exact window selects
        gk_idx = [i for i in live if gk is not None and cols[i].is_float]
        exact = [i for i in live if i not in set(gk_idx)]
        qmap = dict(zip(exact, self.quantiles_batch([(cols[i], packs[i][0], packs[i][1], packs[i][2])
                                                     for i in exact], probs)))
        if gk_idx:
            gq = self.gk_quantiles_batch([cols[i] for i in gk_idx], probs, gk.get('partitions', 1),
                                         gk.get('accuracy', 10000))
            qmap.update({i: (q, False) for i, q in zip(gk_idx, gq)})
        for i in live:                       # candidate slots are no longer needed
            packs[i][2]['cand'] = None
        stats = [None] * len(cols)
        p2_items, p2_idx = [], []
        for i in live:
            qs, fb = qmap[i]
            col, p1 = cols[i], packs[i][0]
            mom = moments(p1, not col.is_float)
            st = NumericStats(count=p1['count'], n_valid=p1['n_valid'], n_nan=p1['n_nan'], n_zero=p1['n_zero'],
                              **mom)
            st.quantiles = qs
            st.fallback_used = fb
            q1, q3 = qs[0.25], qs[0.75]
            k = ks[i]
            hi_t = q3 + k * (q3 - q1)                          # describe.py:222
            lo_t = q1 - k * (q3 - q1)                          # describe.py:223
            st.thresholds = (hi_t, lo_t)
            try:
                edges, width = hist_edges(st.min, st.max, bins)    # describe.py:226 -> :40-45
            except IndexError as e:
                st.error = e
                stats[i] = st
                continue
            st.edges, st.width = edges, width
            p2_items.append((col, st.mean, edges, hi_t, lo_t))
            p2_idx.append(i)
            stats[i] = st
        # columns whose countDistinct takes the partitioning path: pass 2 also
        # does their level-1 count (one column read fewer, single rank or sharded)
        count_ctx = {}
        count32_cols = count32_cols or {}
        for j, i in enumerate(p2_idx):
            if i in count32_cols and not self.comm.sharded:
                # sdp_distinct32's level-1 count on pass 2's read (b1 = -1)
                col = cols[i]
                rpb = sdp.sdp_part_rows_per_block(col.length, 0)
                grid = max(1, -(-col.length // rpb))
                count_ctx[j] = {'d32': True, 'b1': -1, 'hv': None, 'lo': int(count32_cols[i]),
                                'h1': torch.empty(64 * grid, dtype=torch.int32, device=self.device),
                                'hcnt': self._u64(1), 'stats': self._u64(2, zero=True)}
                continue
            if i in group_cols:
                # sharded: group_sharded_batch's level-1 geometry (heavy keys
                # pooled over the ranks, the same on every rank)
                ctx = self._group_prepare_sharded(cols[i]) if self.comm.sharded else \
                    self._group_prepare(cols[i], False)
                if ctx is not None:
                    count_ctx[j] = ctx
        for i, r2 in zip(p2_idx, self.pass2_batch(p2_items, count_ctx)):
            st = stats[i]
            st.mad = r2['abs_dev_sum']
            st.hist_counts = r2['hist']
            st.high_idx = r2['n_high']
            st.low_idx = r2['n_low']
        return stats

    def numeric_pass1(self, col, probs=PROBS):
        plan_dev, plan = self.plan(col, probs)
        local, cand_info = self.pass1(col, plan_dev, plan)
        return self.merge_pass1(local), plan, cand_info

    def numeric_pass1_batch(self, cols, probs=PROBS, minmax_cols=(), byte_cols=()):
        """numeric_pass1 of several columns with the GPU work queued back to
        back: every column's sample + quantile plan, ONE readback of the plans,
        every column's pass 1, ONE readback (one all-gather on a sharded table)
        of the results.  Two host round trips for the whole table instead of two
        per column; results are identical to numeric_pass1 column by column.
        `minmax_cols` (date / timestamp columns, describe.py:233) take pass 1
        without quantile windows in the same launches and readback; with them
        the return value is (packs, [their merged pass-1 results])."""
        if minmax_cols:
            return self._pass1_batch_with_minmax(cols, probs, minmax_cols, byte_cols)
        if not cols:
            return []
        world, sharded = self.comm.world, self.comm.sharded
        ns = max(1, SAMPLE_TOTAL // world)
        s = self._s()
        # every column's struct on the device once: the three sample rounds
        # are one launch each for the whole table
        d_cols = self._h2d(np.frombuffer(bytearray(b''.join(bytes(c.sdp()) for c in cols)), dtype=np.uint8))
        samples = self._u64(len(cols) * ns)
        sdp.sdp_sample_keys_batch(ptr(d_cols), len(cols), ns, ptr(samples), s)
        if sharded:
            # [cols, world * ns]: column i's pooled sample in rank order
            samples = torch.cat([p.view(len(cols), ns) for p in self.comm.allgather(samples)], dim=1).contiguous()
        pr = self._h2d(np.array(list(probs), dtype=np.float64))
        isf = self._h2d(np.array([int(c.is_float) for c in cols], dtype=np.int32))
        psz = ctypes.sizeof(nat.SdpQPlan)
        plans_dev = self._bytes(len(cols) * psz)
        # columns whose sampled keys (evenly spaced rows, in row order: pooled
        # over the ranks in rank order) never decrease may be sorted (ids,
        # timestamps): their countDistinct is verified by one streaming pass
        # (sdp_sorted_distinct) instead of the partitioning pipeline
        mono = self._sample_nondecreasing(samples.view(len(cols), ns * world))
        sdp.sdp_quantile_plan_batch(ptr(samples), ns * world, len(cols), ptr(pr), len(probs), ptr(isf),
                                    ptr(plans_dev), s)
        # narrower windows from a second, 8x larger sample (pooled across ranks
        # like the first): fewer pass-1 candidates and cheaper selects
        ns2 = max(1, SAMPLE2_TOTAL // world)
        # (sharded: always, so every rank takes the same collective path)
        if sharded or min(c.length for c in cols) > SAMPLE_TOTAL:
            s2 = self._u64(len(cols) * ns2)
            sdp.sdp_sample_keys_batch(ptr(d_cols), len(cols), ns2, ptr(s2), s)
            if sharded:
                s2 = torch.cat([p.view(len(cols), ns2) for p in self.comm.allgather(s2)], dim=1).contiguous()
            sdp.sdp_quantile_refine_batch(ptr(s2), ns2 * world, len(cols), ptr(pr), len(probs), ptr(plans_dev), s)
            ns3 = SAMPLE3_TOTAL // world
            if ns3 > ns2 and (sharded or min(c.length for c in cols) > SAMPLE2_TOTAL):
                s3 = self._u64(len(cols) * ns3)
                sdp.sdp_sample_keys_batch(ptr(d_cols), len(cols), ns3, ptr(s3), s)
                if sharded:
                    s3 = torch.cat([p.view(len(cols), ns3) for p in self.comm.allgather(s3)], dim=1).contiguous()
                sdp.sdp_quantile_refine_batch(ptr(s3), ns3 * world, len(cols), ptr(pr), len(probs), ptr(plans_dev), s)
        # heavy-key samples of the columns the partitioning path will group
        # (single rank, >= 64 K rows), sorted on the GPU and read back with the
        # plans; the host finds the heavy keys while pass 1 runs
        # (sharded: every column, PART_SAMPLE / world rows per rank pooled in
        # rank order, the same keys on every rank -- group_sharded's gather)
        hcols = [c for c in cols if sharded or c.length >= (1 << 16)]
        hn_each = PART_SAMPLE // world * world
        hs = None
        if hcols:
            nsr = hn_each // world
            hs = self._u64(len(hcols) * nsr)
            live = [i for i, col in enumerate(hcols) if col.length]
            for i, col in enumerate(hcols):
                if col.length == 0:
                    hs[i * nsr:(i + 1) * nsr].fill_(-1)
            if len(live) == len(hcols):                   # one launch for every column
                d_hc = self._h2d(np.frombuffer(bytearray(b''.join(bytes(c.sdp()) for c in hcols)), dtype=np.uint8))
                sdp.sdp_part_sample_batch(ptr(d_hc), len(hcols), nsr, ptr(hs), s)
            else:
                for i in live:
                    cs = hcols[i].sdp()
                    sdp.sdp_part_sample(ctypes.byref(cs), None, nsr, ptr(hs[i * nsr:]), None, s)
            if sharded:
                hs = torch.cat([p.view(len(hcols), nsr) for p in self.comm.allgather(hs)], dim=1).contiguous()
            sdp.sdp_sort_small_batch(ptr(hs), hn_each, len(hcols), s)
        # the heavy-key samples of the byte columns (value_counts_bytes_batch)
        # ride the same readback; their host work runs while pass 1 does
        bsm = [self._heavy_sample_launch(c, True) for c in byte_cols if c.length >= (1 << 16)]
        bparts = [sm['readback'] if sm['readback'] is not None else sm['h'] for sm in bsm]
        bview = [p.view(torch.uint8) for p in bparts]
        nb_bytes = sum(p.numel() for p in bview)
        raw = torch.cat([plans_dev] + ([hs.view(-1).view(torch.uint8)] if hcols else []) + bview + [mono]).cpu().numpy()
        mono_h = raw[-len(cols):].astype(bool)
        braw = raw[len(raw) - len(cols) - nb_bytes:len(raw) - len(cols)]
        raw = raw[:len(raw) - len(cols) - nb_bytes]
        plans = [nat.SdpQPlan.from_buffer_copy(raw[i * psz:(i + 1) * psz].tobytes()) for i in range(len(cols))]
        if DEBUG_QUANTILE == 'miss':
            for i, p in enumerate(plans):
                for w in range(p.n_windows):
                    p.hi[w] = p.lo[w]
                p.excl_mask = (1 << nat.MAX_WINDOWS) - 1      # (lo, lo): nothing inside, every rank missed
                plans_dev[i * psz:(i + 1) * psz] = self._to_dev(p)
        rsz = ctypes.sizeof(nat.SdpPass1Result)
        res_all = self._bytes(len(cols) * rsz)
        infos = []
        keep_tasks = None
        budget = [CAND_FULL_BUDGET]
        for i, col in enumerate(cols):
            infos.append(self._pass1_launch(col, plans_dev[i * psz:], plans[i], res_all[i * rsz:], budget,
                                            defer=PASS1_BATCH))
        if PASS1_BATCH:
            keep_tasks = self._pass1_run_batch(infos)     # (alive until the pass-1 readback below)
        # (sharded: the flag comes from the pooled sample, the same on every rank)
        sorted_idx = [i for i, c in enumerate(cols)
                      if mono_h[i] and c.kind == 'fixed' and (sharded or c.length >= SORTED_MIN_ROWS)]
        sd = self._u64(4 * max(1, len(sorted_idx)))
        for j, i in enumerate(sorted_idx):
            cs = cols[i].sdp()
            nat.annotate(_label(cols[i], 'sorted'), col_read_bytes(cols[i]))
            sdp.sdp_sorted_distinct(ctypes.byref(cs), ptr(sd[4 * j:]), s)
        if bsm:                                   # (pass 1 is running meanwhile)
            flat, off = braw.view(np.uint64), 0
            for c, sm, p in zip([c for c in byte_cols if c.length >= (1 << 16)], bsm, bparts):
                self._heavy_bytes_pre[id(c)] = self._heavy_keys_finish(sm, flat[off:off + p.numel()])
                off += p.numel()
        if hcols:
            if self._heavy_pre is None:
                self._heavy_pre = {}
                self._near_unique = set()
            hsn = raw[len(cols) * psz:].view(np.uint64).reshape(len(hcols), hn_each)
            for i, col in enumerate(hcols):
                a = hsn[i]
                a = a[:int(np.searchsorted(a, np.uint64(U64)))]      # valid rows sort before UINT64_MAX
                if a.size == 0:
                    self._heavy_pre[id(col)] = None
                    continue
                start = np.flatnonzero(np.concatenate(([True], a[1:] != a[:-1])))
                cnt = np.diff(np.append(start, a.size))
                self._heavy_pre[id(col)] = self._heavy_struct(a[start], cnt)
                if start.size >= 0.9 * a.size:
                    self._near_unique.add(id(col))
        # pass-1 results + sorted checks (+ the date columns' pass 1): one readback
        extra = self._extra_readback
        both = torch.cat([res_all, sd.view(torch.uint8)] + ([extra] if extra is not None else []))
        if not sharded:
            raws = [both.cpu().numpy().tobytes()]
        else:
            raws = [g.cpu().numpy().tobytes() for g in self.comm.allgather(both)]
        if extra is not None:
            tail = len(cols) * rsz + sd.numel() * 8
            self._extra_raws = [r[tail:] for r in raws]
            raws = [r[:tail] for r in raws]
        merged = [merge_pass1_results([nat.SdpPass1Result.from_buffer_copy(r[i * rsz:(i + 1) * rsz]) for r in raws])
                  for i in range(len(cols))]
        off = len(cols) * rsz
        for j, i in enumerate(sorted_idx):
            parts = [np.frombuffer(r[off + 32 * j: off + 32 * j + 32], dtype=np.uint64) for r in raws]
            merged[i]['sorted_distinct'] = merge_sorted_distinct(parts)
        return [(merged[i], plans[i], infos[i]) for i in range(len(cols))]

    def _pass1_batch_with_minmax(self, cols, probs, minmax_cols, byte_cols=()):
        """numeric_pass1_batch plus windowless pass 1 of `minmax_cols`, whose
        results ride the numeric columns' readback (or its all-gather)."""
        rsz = ctypes.sizeof(nat.SdpPass1Result)
        m = len(minmax_cols)
        res = self._bytes(m * rsz)
        plan_dev, plan = self.empty_plan()
        for i, col in enumerate(minmax_cols):
            self._pass1_launch(col, plan_dev, plan, res[i * rsz:])
        self._extra_readback = res
        try:
            packs = self.numeric_pass1_batch(cols, probs, byte_cols=byte_cols) if cols else []
        finally:
            self._extra_readback = None
        raws = self._extra_raws if cols else None
        if raws is None:                                   # no numeric columns: read back alone
            raws = [res.cpu().numpy().tobytes()] if not self.comm.sharded else \
                [g.cpu().numpy().tobytes() for g in self.comm.allgather(res)]
        mm = [merge_pass1_results([nat.SdpPass1Result.from_buffer_copy(r[i * rsz:(i + 1) * rsz]) for r in raws])
              for i in range(m)]
        return packs, mm

    _extra_readback = None
    _extra_raws = None

    @staticmethod
    def _sample_nondecreasing(samp):
        """[cols, m] sampled keys in row order (UINT64_MAX = null/NaN row) ->
        uint8 [cols]: 1 where the valid keys never decrease (at least 2)."""
        valid = samp != -1
        x = samp ^ (-(1 << 63))                      # unsigned key order as signed order
        x = torch.where(valid, x, torch.full_like(x, -(1 << 63)))
        run = torch.cummax(x, dim=1).values
        down = (valid & (x < run)).any(dim=1)
        return (~down & (valid.sum(dim=1) >= 2)).to(torch.uint8)

    def minmax_pass(self, col):
        """count / min / max of a date or timestamp column (describe.py:233)."""
        plan_dev, plan = self.empty_plan()
        local, _ = self.pass1(col, plan_dev, plan)
        return self.merge_pass1(local)

    # ==========================================================================
    # distinct counts and value counts
    # ==========================================================================
    def _table(self, capacity, bytes_keys, with_counts=True):
        slots = self._u64(capacity)
        counts = self._u64(capacity) if with_counts else None
        sdp.sdp_table_clear(ptr(slots), ptr(counts), capacity, int(bytes_keys), self._s())
        return slots, counts

    # -- two-level hash partitioning (sdp_part.hip) ------------------------------
    def _records(self, n, isb):
        keep = [self._u64(max(n, 1))]
        if isb:
            keep += [self._u64(max(n, 1)), self._u64(max(n, 1))]
        r = nat.SdpRecords(keep[0].data_ptr(), keep[1].data_ptr() if isb else None,
                           keep[2].data_ptr() if isb else None)
        return r, keep

    @staticmethod
    def _l2b_ok(isb, b2, heavy=False):
        """sdp_part_l2_blocks takes this level 2 (<= 1024 sub-buckets of fixed
        keys, <= 512 of byte keys: the LDS lines of one workgroup) -- but not
        for fixed keys with heavy keys in the sample: a skewed column's copies
        land in whole groups, so many sub-buckets overflow their runs and the
        block dedup reads them through the lists (i64_zipf: count + scatter +
        dedup 6.5 ms counted vs 9.7 ms in blocks; near-unique and byte columns
        gain, profiles/r06m_*)."""
        if heavy and not isb:
            return False
        return L2_BLOCKS and 1 <= b2 and (1 << b2) <= (512 if isb else 1024)

    L2B_WG = 256                       # persistent workgroups of sdp_part_l2_blocks (one per CU)

    def _l2_blocks(self, r1, isb, b1, b2, seg_lo, seg_hi, seg_bucket, nbk):
        """Level 2 of nbk level-1 buckets into blocks (sdp_part_l2_blocks): the
        records of bucket i are the segments [seg_lo, seg_hi) of r1 whose
        seg_bucket is i (host arrays, a bucket's segments consecutive).  No
        count pass, no scan: one workgroup per bucket at a time, buckets dealt
        to the workgroups by size (largest first, snake order).  Returns
        (records, their tensors, SdpBlocks, the block tensors)."""
        seg_lo = np.asarray(seg_lo, dtype=np.int64)
        seg_hi = np.asarray(seg_hi, dtype=np.int64)
        seg_bucket = np.asarray(seg_bucket, dtype=np.int64)
        nb2 = 1 << b2
        sizes = np.bincount(seg_bucket, weights=seg_hi - seg_lo, minlength=nbk).astype(np.int64)
        # sub-bucket runs of mean + 4 sigma records (a near-unique column's
        # sub-buckets practically never spill into overflow blocks); the
        # overflow space covers every record, so nothing can overflow
        mean = sizes / float(nb2)
        R = np.ceil((mean + 4.0 * np.sqrt(mean) + 16.0) / L2_BLOCK).astype(np.int64)
        nblk = (nb2 * R + -(-sizes // L2_BLOCK) + 8 + 7) // 8 * 8  # regions on 64-byte lines of bmeta
        rbase = np.zeros(nbk + 1, dtype=np.int64)
        rbase[1:] = np.cumsum(nblk)
        total = int(rbase[-1])
        if total >= (1 << 32):
            raise nat.NativeError('l2_blocks: %d blocks' % total)
        G = min(self.L2B_WG, nbk)
        rank = np.empty(nbk, dtype=np.int64)
        rank[np.argsort(-sizes, kind='stable')] = np.arange(nbk)
        rnd, pos = rank // G, rank % G
        wg = np.where(rnd % 2 == 0, pos, G - 1 - pos)             # snake: round-robin, reversed every round
        # segments in (workgroup, bucket rank, segment) order
        nseg = len(seg_lo)
        order = np.lexsort((np.arange(nseg), rank[seg_bucket], wg[seg_bucket]))
        sb = seg_bucket[order]
        first = np.ones(nseg, dtype=bool)
        first[1:] = sb[1:] != sb[:-1]
        last = np.ones(nseg, dtype=bool)
        last[:-1] = sb[1:] != sb[:-1]
        tab = np.empty((nseg, 4), dtype=np.int64)
        tab[:, 0] = seg_lo[order]
        tab[:, 1] = seg_hi[order]
        tab[:, 2] = sb
        tab[:, 3] = rbase[sb] | (first.astype(np.int64) << 32) | (last.astype(np.int64) << 33) | (R[sb] << 40)
        soff = np.zeros(G + 1, dtype=np.int64)
        soff[1:] = np.cumsum(np.bincount(wg[sb], minlength=G))
        dt = self._h2d(np.concatenate([tab.reshape(-1), soff]))
        rf, keepf = self._records(total * L2_BLOCK, isb)
        bmeta = self._u64(total)
        # (the dedup kernels read a batch's list entries in one load: padding)
        lst = torch.empty(total + 32, dtype=torch.int32, device=self.device)
        fc = torch.empty(nbk * nb2 * nat.L2_DESC_W, dtype=torch.int32, device=self.device)
        blk = nat.SdpBlocks(fc.data_ptr(), lst.data_ptr())
        if DEBUG_BOUNDS:                   # (test builds: the capacities the bounds checks use)
            sdp.sdp_debug_bounds(total * L2_BLOCK, total + 32, None, 0)
        sdp.sdp_part_l2_blocks(ctypes.byref(r1), int(isb), ptr(dt), ctypes.c_void_p(dt.data_ptr() + 8 * tab.size), G,
                               b1, b2, ctypes.byref(rf), ptr(bmeta), ctypes.byref(blk), self._s())
        del bmeta, dt
        return rf, keepf, blk, (fc, lst)

    def _heavy_keys(self, col, isb, gather=False):
        """Keys seen >= HEAVY_MIN times in an evenly spaced sample: counted
        outside the partitions (describe.py:251's hot groups).  gather=True
        (fixed keys of a sharded table): the samples of all ranks are pooled,
        so every rank picks the same heavy keys."""
        if not isb and gather == self.comm.sharded and self._heavy_pre and id(col) in self._heavy_pre:
            return self._heavy_pre.pop(id(col))        # sampled with pass 1 (numeric_pass1_batch)
        smp = self._heavy_sample_launch(col, isb, gather)
        if smp['readback'] is not None:
            host = smp['readback'].cpu().numpy().view(np.uint64)
        else:
            host = smp['h'].cpu().numpy().view(np.uint64)
        return self._heavy_keys_finish(smp, host)

    def _heavy_sample_launch(self, col, isb, gather=False):
        """Queue the heavy-key sample of `col` (no readback)."""
        ns = min(PART_SAMPLE_BYTES if isb else PART_SAMPLE, max(col.length, 1))
        if gather and self.comm.sharded:
            ns = max(1, min(PART_SAMPLE // self.comm.world, col.length))   # pooled: PART_SAMPLE in all
        s = self._s()
        h = self._u64(ns)
        if col.length == 0:
            h.fill_(-1)
            keep = None
        elif isb:
            rec, keep = self._records(ns, True)
            sdp.sdp_part_sample(None, ctypes.byref(col.sdp_bytes()), ns, ptr(h), ctypes.byref(rec), s)
        else:
            keep = None
            sdp.sdp_part_sample(ctypes.byref(col.sdp()), None, ns, ptr(h), None, s)
        if gather and self.comm.sharded:
            h = torch.cat(self.comm.allgatherv(h))
        # sample hashes (and byte-key metas) leave the device in one piece
        readback = torch.cat([h, keep[2][:ns]]) if (isb and keep is not None) else None
        return {'h': h, 'keep': keep, 'ns': ns, 'isb': isb, 'readback': readback}

    def _heavy_keys_batch(self, cols):
        """_heavy_keys of several byte columns with ONE readback of all samples."""
        smps = [self._heavy_sample_launch(c, True) for c in cols]
        parts = [sm['readback'] if sm['readback'] is not None else sm['h'] for sm in smps]
        if not parts:
            return []
        flat = torch.cat(parts).cpu().numpy().view(np.uint64)
        out, off = [], 0
        for sm, p in zip(smps, parts):
            out.append(self._heavy_keys_finish(sm, flat[off:off + p.numel()]))
            off += p.numel()
        return out

    def _heavy_keys_finish(self, smp, host):
        """Heavy keys from the host copy of a sample (see _heavy_sample_launch)."""
        h, keep, ns, isb = smp['h'], smp['keep'], smp['ns'], smp['isb']
        meta = None
        if isb and keep is not None:
            hn, meta = host[:h.numel()], host[h.numel():]
        else:
            hn = host
        pos = np.nonzero(hn != np.uint64(U64))[0]
        n_valid = pos.size
        if isb and pos.size:
            pos = pos[(meta[pos] >> np.uint64(40)) <= np.uint64(16)]
        if pos.size == 0:
            return None
        u, first, cnt = np.unique(hn[pos], return_index=True, return_counts=True)
        hv = self._heavy_struct(u, cnt, first, pos, keep, isb, meta)
        if hv is not None:        # sampled share of rows that become partition records
            hv['rec_frac'] = (n_valid - hv['heavy_rows']) / float(len(hn))
            hv['ns'] = len(hn)
        return hv

    def _heavy_struct(self, u, cnt, first=None, pos=None, keep=None, isb=False, meta=None):
        """Heavy keys (>= HEAVY_MIN sample occurrences, at most HEAVY_MAX by
        count) from the sample's distinct hashes u (ascending) and counts.
        Host copies of the hashes (and byte-key metas) stay in the dict, so the
        group assembly needs no readback of them."""
        sel = np.nonzero(cnt >= HEAVY_MIN)[0]
        if sel.size == 0:
            return None
        # at most HEAVY_MAX keys (HEAVY_MAX_REC for byte keys: the records kernel
        # holds them; the other byte kernels take the first HEAVY_MAX, _hv_cap),
        # the most frequent first
        cap = nat.HEAVY_MAX_REC if isb else nat.HEAVY_MAX
        sel = sel[np.argsort(-cnt[sel], kind='stable')[:cap]]
        hv = {'h': self._h2d(u[sel].view(np.int64).copy()), 'n': int(sel.size),
              'h_host': [int(x) for x in u[sel].tolist()], 'heavy_rows': int(cnt[sel].sum()),
              'cnt_host': [int(x) for x in cnt[sel].tolist()]}
        if isb:
            rows = pos[first[sel]]
            hv['meta_host'] = [int(x) for x in meta[rows].tolist()]
            idx = self._h2d(rows.astype(np.int64))
            hv['k0'], hv['k1'], hv['meta'] = keep[0][idx].contiguous(), keep[1][idx].contiguous(), \
                keep[2][idx].contiguous()
        st = nat.SdpHeavy(hv['h'].data_ptr(), hv['k0'].data_ptr() if isb else None,
                          hv['k1'].data_ptr() if isb else None, hv['meta'].data_ptr() if isb else None, hv['n'], 0)
        hv['struct'] = st
        return hv

    def group(self, col, with_counts, dense=True):
        """Exact groups of a column by two-level hash partitioning with exact
        offsets (sdp_part.hip).  Returns a tab dict (dense (key, count) group
        arrays when counts are needed), or None when the column needs the exact
        global-table path (64-bit hash collision between different strings, or
        a final bucket larger than its LDS table).  Two host readbacks: the
        level-1 bucket starts, then the group statistics."""
        ctx = self._group_begin(col, with_counts)
        if ctx is None:
            return None
        self._group_middle(ctx, ctx['bsn_dev'].cpu().numpy().astype(np.int64))
        return self._group_end(ctx, self._host_u64(ctx['stats_dev']), dense)

    def group_batch(self, cols):
        """group(col, with_counts=False, dense=False) -- countDistinct
        (describe.py:143) -- of several columns with two host readbacks in
        all: every column's level-1 count, one readback of every bucket-start
        array, every column's scatters and de-duplication queued back to back
        (record buffers recycled on the stream between columns), one readback
        of every column's group statistics.  None where group() returns None."""
        ctxs = []
        for c in cols:
            pre = self._counted.pop(id(c), None)           # counted by pass 2 (sdp_pass2_count)
            if pre is not None and pre.get('d32'):         # a 32-bit-path count: not this path's
                pre = None
            if pre is None:
                pre = self._group_prepare(c, False)
                if pre is not None:
                    self._group_count(pre)
            ctxs.append(pre)
        live = [c for c in ctxs if c is not None]
        if not live:
            return [None] * len(cols)
        # wide tables: columns of one geometry share one scan of their level-1
        # counts (global record positions: column c's records start where
        # column c-1's end) and their level-1 scatter, level-2 and
        # de-duplication launches (_group_middle_fused); the rest one by one
        fuse, single = self._fusable(live)
        for grp in fuse:
            self._group_scan_shared([live[i] for i in grp])
        for i in single:
            self._group_scan(live[i])
        flat = torch.cat([c['bsn_dev'] for c in live]).cpu().numpy().astype(np.int64)
        off, bsns = 0, []
        for c in live:
            m = c['bsn_dev'].numel()
            bsns.append(flat[off:off + m])
            off += m
        for grp in fuse:
            self._group_middle_fused([live[i] for i in grp], [bsns[i] for i in grp])
        for i in single:
            self._group_middle(live[i], bsns[i])
        sizes = [c['stats_dev'].numel() for c in live]
        allst = self._host_u64(torch.cat([c['stats_dev'] for c in live]))
        out, off, it = [], 0, iter(zip(live, sizes))
        for c in ctxs:
            if c is None:
                out.append(None)
                continue
            ctx, m = next(it)
            out.append(self._group_end(ctx, allst[off:off + m], False))
            off += m
        return out

    _NO_HV = object()

    def _group_prepare(self, col, with_counts, hv=_NO_HV):
        """Geometry and buffers of the two-level partitioning of `col` (None
        when the column needs more than 20 hash bits of buckets); `hv` = heavy
        keys already sampled (_heavy_keys_batch)."""
        isb = col.kind == 'bytes'
        with_counts = with_counts or isb
        n = col.length
        target = sdp.sdp_part_bucket_target(int(isb), int(with_counts))
        if hv is Engine._NO_HV:
            hv = self._heavy_keys(col, isb)
        if isb and not BYTES_ONE_READ:
            hv = self._hv_cap(hv, nat.HEAVY_MAX)       # the row kernels' LDS tables hold fewer
        while True:
            n_rec = n
            if isb and hv is not None and 'rec_frac' in hv:
                # byte columns: size the buckets for the records the sample predicts
                # (heavy keys never become records), with margin; fewer hash bits
                # mean longer runs per bucket in both scatters
                n_rec = min(n, int(n * (1.25 * hv['rec_frac'] + 0.02)) + 1)
            total_bits = max(0, math.ceil(math.log2(max(1.0, n_rec / target))))
            b1 = min(10, (total_bits + 1) // 2)
            one_read = isb and BYTES_ONE_READ and b1 > 0
            if not isb or one_read or hv is None or hv['n'] <= nat.HEAVY_MAX:
                break
            hv = self._hv_cap(hv, nat.HEAVY_MAX)       # b1 == 0: the row kernels take the bytes
        large = False
        if total_bits > 20 and not isb and not with_counts:
            # > 2^30 rows: 4x larger final buckets on the workgroup-table kernel
            total_bits = max(20, math.ceil(math.log2(max(1.0, n / (4 * target)))))
            large = True
            b1 = min(10, (total_bits + 1) // 2)
        b2 = total_bits - b1
        if b2 > 10:
            return None
        nb1, nb2 = 1 << b1, 1 << b2
        rpb = sdp.sdp_part_rows_per_block(n, int(isb))
        grid = max(1, -(-n // rpb))
        if one_read:
            grid = sdp.sdp_part_records_chunks(n)           # one level-1 histogram per wave strip
        return {'col': col, 'isb': isb, 'with_counts': with_counts, 'large': large, 'b1': b1, 'b2': b2,
                'nb1': nb1, 'nb2': nb2, 'stats': self._u64(68, zero=True), 'cs': None if isb else col.sdp(),
                'bc': col.sdp_bytes() if isb else None, 'hv': hv,
                'hcnt': self._u64(max(hv['n'] if hv else 1, 1), zero=True), 'grid': grid,
                'h1': torch.empty(nb1 * grid, dtype=torch.int32, device=self.device),
                'rb': col_read_bytes(col), 'recw': 24 if isb else 8,
                'one_read': one_read}

    @staticmethod
    def _hv_cap(hv, cap):
        """The first `cap` heavy keys of hv (the most frequent: _heavy_struct
        orders them by sample count).  Rows of the dropped keys simply become
        partition records; the groups come out the same."""
        if hv is None or hv['n'] <= cap:
            return hv
        out = dict(hv)
        out['n'] = cap
        out['h_host'] = hv['h_host'][:cap]
        if 'meta_host' in hv:
            out['meta_host'] = hv['meta_host'][:cap]
        if 'cnt_host' in hv:
            out['cnt_host'] = hv['cnt_host'][:cap]
            out['heavy_rows'] = int(sum(out['cnt_host']))
            if 'rec_frac' in hv:
                out['rec_frac'] = hv['rec_frac'] + (hv['heavy_rows'] - out['heavy_rows']) / float(hv['ns'])
        st = hv['struct']
        out['struct'] = nat.SdpHeavy(st.d_h, st.d_k0, st.d_k1, st.d_meta, cap, 0)
        return out

    def _group_count(self, ctx):
        """Level-1 bucket counts (sdp_part_rows phase 0).  Byte columns
        (one_read): the strings are read once, into compacted per-strip
        records that _group_middle scatters (sdp_part_rows_records)."""
        col, isb, hv = ctx['col'], ctx['isb'], ctx['hv']
        if ctx['one_read']:
            r0, keep0 = self._records(col.length, True)
            chunks = torch.empty((ctx['grid'], 4), dtype=torch.int64, device=self.device)
            nat.annotate(_label(col, 'records'), ctx['rb'])
            sdp.sdp_part_rows_records(ctypes.byref(ctx['bc']), ctypes.byref(hv['struct']) if hv else None,
                                      ctx['b1'], ptr(ctx['h1']), ptr(chunks), ctypes.byref(r0), ptr(ctx['hcnt']),
                                      ptr(ctx['stats']), self._s())
            ctx['rec_key'] = 'sdp_part_rows_records[%s]' % _label(col, 'records')
            ctx['rec_idx'] = nat.recorded_index(ctx['rec_key'])
            ctx.update({'r0': r0, 'keep0': keep0, 'chunks0': chunks})
            return
        nat.annotate(_label(col, 'count'), ctx['rb'])
        sdp.sdp_part_rows(self._gref(ctx), ctypes.byref(ctx['bc']) if isb else None,
                          ctypes.byref(hv['struct']) if hv else None, ctx['b1'], 0, ptr(ctx['h1']), None, None,
                          ptr(ctx['hcnt']), ptr(ctx['stats']), self._s())

    def _group_scan(self, ctx):
        o1 = self._scan(ctx['h1'])
        del ctx['h1']
        nb1, grid = ctx['nb1'], ctx['grid']
        ctx['o1'] = o1
        ctx['bsn_dev'] = torch.cat([o1[0:nb1 * grid:grid], o1[-1:]])     # record count + L1 bucket starts
        return ctx

    def _group_begin(self, col, with_counts):
        """Level-1 bucket counts of `col` and their scan (no readback)."""
        ctx = self._group_prepare(col, with_counts)
        if ctx is None:
            return None
        self._group_count(ctx)
        return self._group_scan(ctx)

    @staticmethod
    def _gref(ctx):
        return None if ctx['isb'] else ctypes.byref(ctx['cs'])

    def _group_middle(self, ctx, bsn):
        """Level-1 scatter, level-2 count/scan/scatter and the LDS
        de-duplication, all queued; `bsn` = the host copy of bsn_dev."""
        s = self._s()
        isb, with_counts, large = ctx['isb'], ctx['with_counts'], ctx['large']
        b1, b2, nb1, nb2, grid = ctx['b1'], ctx['b2'], ctx['nb1'], ctx['nb2'], ctx['grid']
        col, hv, hcnt, stats, o1 = ctx['col'], ctx['hv'], ctx['hcnt'], ctx['stats'], ctx['o1']
        rb, recw = ctx['rb'], ctx['recw']
        cref = self._gref(ctx)
        bref = ctypes.byref(ctx['bc']) if isb else None
        hvref = ctypes.byref(hv['struct']) if hv else None
        nrec = int(bsn[-1])
        r1, keep1 = self._records(nrec, isb)
        if ctx.get('one_read'):
            # the records kernel's compulsory output: its nrec 24-byte records
            nat.annotate_output(ctx['rec_key'], ctx['rec_idx'], nrec * recw)
            if nrec:                  # level-1 scatter of the compacted strip records (sequential 24-byte reads)
                nat.annotate('bytes/l1scatter', 2 * nrec * recw)
                sdp.sdp_part_recs(ctypes.byref(ctx['r0']), 1, ptr(ctx['chunks0']), grid, 0, b1, 1, None, ptr(o1),
                                  ctypes.byref(r1), s)
            del ctx['r0'], ctx['keep0'], ctx['chunks0']
        elif nrec:
            nat.annotate(_label(col, 'scatter'), rb + nrec * recw)
            sdp.sdp_part_rows(cref, bref, hvref, b1, 1, None, ptr(o1), ctypes.byref(r1), ptr(hcnt), ptr(stats), s)
        # level 2: each L1 bucket -> nb2 sub-buckets, chunk by chunk
        bstarts = o1[0:nb1 * grid:grid]
        blk = None
        if b2 == 0 or nrec == 0:
            starts = torch.cat([bstarts, o1[-1:]]) if b2 == 0 else self._u64(nb1 * nb2 + 1, zero=True)
            rf, keepf = r1, keep1
        elif self._l2b_ok(isb, b2, bool(hv and hv['n'])):
            nat.annotate(('bytes' if isb else 'u64') + '/l2blocks', 2 * nrec * recw)
            rf, keepf, blk, blk_keep = self._l2_blocks(r1, isb, b1, b2, bsn[:-1], bsn[1:], np.arange(nb1), nb1)
            del keep1, r1
            starts = None
        else:
            bs = bsn
            sizes = np.diff(bs)
            nch = -(-sizes // PART_CHUNK)
            k0 = np.concatenate([[0], np.cumsum(nch)[:-1]]).astype(np.int64)
            K = int(nch.sum())
            bof = np.repeat(np.arange(nb1), nch)
            j = np.arange(K, dtype=np.int64) - k0[bof]
            ch = np.empty((K, 4), dtype=np.int64)
            ch[:, 0] = bs[bof] + j * PART_CHUNK
            ch[:, 1] = np.minimum(bs[bof + 1], ch[:, 0] + PART_CHUNK)
            ch[:, 2] = nb2 * k0[bof] + j
            ch[:, 3] = nch[bof]
            chunks = self._h2d(ch)
            h2 = torch.empty(nb2 * K, dtype=torch.int32, device=self.device)
            nat.annotate(('bytes' if isb else 'u64') + '/count', nrec * recw)
            sdp.sdp_part_recs(ctypes.byref(r1), int(isb), ptr(chunks), K, b1, b2, 0, ptr(h2), None, None, s)
            o2 = self._scan(h2)
            rf, keepf = self._records(nrec, isb)
            nat.annotate(('bytes' if isb else 'u64') + '/scatter', 2 * nrec * recw)
            sdp.sdp_part_recs(ctypes.byref(r1), int(isb), ptr(chunks), K, b1, b2, 1, None, ptr(o2),
                              ctypes.byref(rf), s)
            del keep1, r1, h2
            sidx = (nb2 * k0[:, None] + np.arange(nb2)[None, :] * nch[:, None]).reshape(-1)
            sidx = np.append(sidx, nb2 * K)
            starts = o2[self._h2d(sidx)].contiguous()
        nfinal = nb1 * nb2
        ngroups = torch.zeros(nfinal, dtype=torch.int32, device=self.device)
        out_key = out_cnt = None
        if with_counts:
            nout = keepf[0].numel() if blk is not None else max(nrec, 1)
            out_key, out_cnt = self._u64(nout), self._u64(nout)
        if nrec:
            nat.annotate('bytes' if isb else ('u64/counts' if with_counts else 'u64'), nrec * recw)
            direct = 4 if (not isb and not with_counts and not large and id(col) in self._near_unique) else 0
            mode = int(with_counts) | (2 if large else 0) | direct
            if blk is not None:
                sdp.sdp_part_dedup_blocks(ctypes.byref(rf), int(isb), bref, ctypes.byref(blk), nfinal, mode,
                                          ptr(out_key), ptr(out_cnt), ptr(ngroups), ptr(stats), s)
            else:
                sdp.sdp_part_dedup(ctypes.byref(rf), int(isb), bref, ptr(starts), nfinal, mode,
                                   ptr(out_key), ptr(out_cnt), ptr(ngroups), ptr(stats), s)
        del keepf, rf
        ctx.update({'starts': starts, 'ngroups': ngroups, 'out_key': out_key, 'out_cnt': out_cnt, 'nfinal': nfinal,
                    'blk': blk, 'blk_keep': blk_keep if blk is not None else None})
        del ctx['o1'], ctx['bsn_dev']
        ctx['stats_dev'] = torch.cat([stats, hcnt[:hv['n']]]) if hv else stats

    # dtypes sdp_part_rows_batch dispatches (sdp_part.hip; bit-packed bools excluded)
    ROWS_BATCH_DTYPES = (nat.F64, nat.F32, nat.I64, nat.I32, nat.I16, nat.I8, nat.U64, nat.U32, nat.U16, nat.U8)
    FUSE_MIN_COLS = 8                  # columns of one geometry before their stages are fused
    FUSE_BYTES = 32 << 30              # two 8-byte record buffers of a fused group alive at once
    FUSE_MAX_RECS = 1 << 26            # larger columns fill the GPU alone (and recycle their buffers)

    def _fusable(self, ctxs):
        """Partition group_batch's contexts (before their scans) into groups
        whose stages run fused (fixed keys, distinct only, one (b1, b2), dtype
        and DIRECT mode, a level 2, <= FUSE_MAX_RECS rows each, two 8-byte
        record buffers under FUSE_BYTES) and singles."""
        by, single = {}, []
        for i, c in enumerate(ctxs):
            n = c['col'].length
            if (c['isb'] or c['with_counts'] or c['large'] or c['b2'] == 0 or n == 0 or n > self.FUSE_MAX_RECS
                    or c['col'].dtype not in self.ROWS_BATCH_DTYPES):
                single.append(i)
            else:
                by.setdefault((c['b1'], c['b2'], c['col'].dtype, id(c['col']) in self._near_unique), []).append(i)
        fuse = []
        for key, idx in by.items():
            if len(idx) < self.FUSE_MIN_COLS:
                single += idx
                continue
            grp, held = [], 0
            for i in idx:
                need = 16 * ctxs[i]['col'].length
                if grp and held + need > self.FUSE_BYTES:
                    fuse.append(grp)
                    grp, held = [], 0
                grp.append(i)
                held += need
            fuse.append(grp)
        single += [g[0] for g in fuse if len(g) == 1]
        return [g for g in fuse if len(g) > 1], sorted(single)

    def _group_scan_shared(self, ctxs):
        """ONE exclusive scan of the concatenated level-1 counts of `ctxs`
        (bucket-major per column): o1 / bsn_dev of column c then hold global
        positions in the group's shared record buffer."""
        lens = [c['h1'].numel() for c in ctxs]
        O = self._scan(torch.cat([c.pop('h1') for c in ctxs]))
        off = 0
        for c, m in zip(ctxs, lens):
            o1 = O[off:off + m + 1]
            nb1, grid = c['nb1'], c['grid']
            c['o1'] = o1
            c['bsn_dev'] = torch.cat([o1[0:nb1 * grid:grid], o1[-1:]])
            off += m
        ctxs[0]['_shared_scan'] = O

    def _group_middle_fused(self, ctxs, bsns):
        """_group_middle of several fixed-key, distinct-only columns of one
        (b1, b2): their level-1 scatters write into one record buffer (column c
        from base_c), the level-2 chunk tables are concatenated (histogram
        slots offset per column), so ONE level-2 count, ONE scan, ONE level-2
        scatter, ONE gather of final-bucket starts and ONE de-duplication launch
        (per-bucket group counts, summed per column on the device) serve them
        all.  Each context then carries the same statistics vector as
        _group_middle leaves."""
        s = self._s()
        b1, b2 = ctxs[0]['b1'], ctxs[0]['b2']
        nb1, nb2 = 1 << b1, 1 << b2
        # bsns hold global positions (_group_scan_shared): column c's records
        # are [bs_c[0], bs_c[-1]) of the shared buffer
        total = int(bsns[-1][-1])
        r1, keep1 = self._records(total, False)
        tasks = (nat.SdpRowsTask * len(ctxs))()
        max_grid = max(c['grid'] for c in ctxs)
        for j, ctx in enumerate(ctxs):
            hv = ctx['hv']
            # the task table lives in device memory, so the checks sdp_part_rows
            # makes on its arguments are made here (sdp.h, sdp_part_rows_batch)
            if ctx['col'].values.data_ptr() % 16 or (hv is not None and hv['n'] > nat.HEAVY_MAX) \
                    or ctx['grid'] > max_grid or max_grid > nat.PART_MAX_GRID:
                raise nat.NativeError('part_rows_batch: task %d fails the sdp_part_rows checks' % j)
            tasks[j] = nat.SdpRowsTask(ctx['cs'], hv['struct'] if hv else nat.SdpHeavy(None, None, None, None, 0, 0),
                                       ctx['o1'].data_ptr(), keep1[0].data_ptr(),
                                       sdp.sdp_part_rows_per_block(ctx['col'].length, 0), b1, ctx['grid'])
        d_tasks = self._h2d(np.frombuffer(bytearray(bytes(tasks)), dtype=np.uint8))
        nat.annotate(_label(ctxs[0]['col'], 'scatter_batch'), sum(c['rb'] for c in ctxs) + total * 8)
        sdp.sdp_part_rows_batch(ptr(d_tasks), len(ctxs), ctxs[0]['col'].dtype, max_grid, s)
        shared = ctxs[0].pop('_shared_scan', None)
        for ctx in ctxs:
            del ctx['o1'], ctx['bsn_dev']
        del shared
        nfinal = nb1 * nb2
        nf = nfinal * len(ctxs)
        if self._l2b_ok(False, b2, any(c['hv'] and c['hv']['n'] for c in ctxs)):
            # level 2 of every column's level-1 buckets into blocks: one
            # workgroup per (column, bucket), no count pass
            bst = np.concatenate([bs[:-1] for bs in bsns] + [[total]]).astype(np.int64)
            nat.annotate('u64/l2blocks', 2 * total * 8)
            rf, keepf, blk, blk_keep = self._l2_blocks(r1, False, b1, b2, bst[:-1], bst[1:], np.arange(len(bst) - 1),
                                                       len(bst) - 1)
            del keep1, r1
            ngroups = torch.empty(nf, dtype=torch.int32, device=self.device)
            stats = self._u64(68, zero=True)
            nat.annotate('u64', total * 8)
            direct = 4 if id(ctxs[0]['col']) in self._near_unique else 0
            sdp.sdp_part_dedup_blocks(ctypes.byref(rf), 0, None, ctypes.byref(blk), nf, direct, None, None,
                                      ptr(ngroups), ptr(stats), s)
            del keepf, rf, blk_keep
            self._fused_stats(ctxs, ngroups, stats, nfinal)
            return
        base = np.array([bs[0] for bs in bsns] + [total], dtype=np.int64)
        bsns = [bs - bs[0] for bs in bsns]                      # column-local bucket starts
        # every column's level-2 chunk table at once ([column, L1 bucket] arrays):
        # chunks of <= PART_CHUNK records, ordered (column, bucket, chunk); the
        # histogram slot of (column, bucket, sub-bucket, chunk) is
        # hb[column] + nb2 * k0 + sub * nch + j
        C = len(ctxs)
        bs = np.stack(bsns)                                          # [C, nb1 + 1], column-local
        sizes = np.diff(bs, axis=1)
        nch = -(-sizes // PART_CHUNK)                                # [C, nb1]
        Kc = nch.sum(1)
        k0 = np.cumsum(nch, axis=1) - nch                            # column-local first chunk of each bucket
        hbc = np.concatenate([[0], np.cumsum(nb2 * Kc)[:-1]]).astype(np.int64)
        hb = int((nb2 * Kc).sum())
        flat_n = nch.reshape(-1)
        cb = np.repeat(np.arange(C * nb1), flat_n)                   # (column, bucket) of every chunk
        first = np.cumsum(flat_n) - flat_n
        j = np.arange(int(flat_n.sum()), dtype=np.int64) - first[cb]
        col_of, b_of = cb // nb1, cb % nb1
        start0 = base[col_of] + bs[col_of, b_of] + j * PART_CHUNK
        ch = np.empty((len(cb), 4), dtype=np.int64)
        ch[:, 0] = start0
        ch[:, 1] = np.minimum(base[col_of] + bs[col_of, b_of + 1], start0 + PART_CHUNK)
        ch[:, 2] = hbc[col_of] + nb2 * k0[col_of, b_of] + j
        ch[:, 3] = nch[col_of, b_of]
        sidx = (hbc[:, None, None] + nb2 * k0[:, :, None]
                + np.arange(nb2)[None, None, :] * nch[:, :, None]).reshape(-1)
        chunks = self._h2d(ch)
        h2 = torch.empty(hb, dtype=torch.int32, device=self.device)
        nat.annotate('u64/count', total * 8)
        sdp.sdp_part_recs(ctypes.byref(r1), 0, ptr(chunks), len(ch), b1, b2, 0, ptr(h2), None, None, s)
        o2 = self._scan(h2)
        rf, keepf = self._records(total, False)
        nat.annotate('u64/scatter', 2 * total * 8)
        sdp.sdp_part_recs(ctypes.byref(r1), 0, ptr(chunks), len(ch), b1, b2, 1, None, ptr(o2), ctypes.byref(rf), s)
        del keep1, r1, h2
        starts = o2[self._h2d(np.append(sidx, hb))].contiguous()
        ngroups = torch.empty(nf, dtype=torch.int32, device=self.device)
        stats = self._u64(68, zero=True)
        nat.annotate('u64', total * 8)
        direct = 4 if id(ctxs[0]['col']) in self._near_unique else 0
        sdp.sdp_part_dedup(ctypes.byref(rf), 0, None, ptr(starts), nf, direct, None, None, ptr(ngroups), ptr(stats), s)
        del keepf, rf
        self._fused_stats(ctxs, ngroups, stats, nfinal)

    @staticmethod
    def _fused_stats(ctxs, ngroups, stats, nfinal):
        """Every fused column's statistics vector from the shared dedup's
        per-bucket group counts and flags."""
        per_col = ngroups.view(len(ctxs), nfinal).to(torch.int64).sum(1)
        for ci, ctx in enumerate(ctxs):
            st = ctx['stats']
            st[4] += per_col[ci]                     # (the count pass left 4..67 at zero)
            st[3] |= stats[3]                        # a full table anywhere: every fused column recounts
            hv = ctx['hv']
            ctx['stats_dev'] = torch.cat([st, ctx['hcnt'][:hv['n']]]) if hv else st
            ctx.update({'starts': None, 'ngroups': None, 'out_key': None, 'out_cnt': None, 'nfinal': nfinal})

    def _group_end(self, ctx, both, dense):
        """The tab dict from the host copy of stats_dev (see group)."""
        s = self._s()
        isb, with_counts, col, hv = ctx['isb'], ctx['with_counts'], ctx['col'], ctx['hv']
        st, hc = both[:68], both[68:]
        if st[2] or st[3]:
            return None
        groups_local = sum(st[4:68])
        special = st[1]
        heavy_sel = [i for i, c in enumerate(hc) if c]
        total = groups_local + (1 if special else 0) + len(heavy_sel)
        tab = {'bytes': isb, 'dense': True, 'rows': st[0], 'max_key_rows': 0, 'col': col,
               'groups': total, 'groups_local': total}
        if dense and with_counts:
            starts, ngroups, nfinal = ctx['starts'], ctx['ngroups'], ctx['nfinal']
            keys = self._u64(max(total, 1))
            counts = self._u64(max(total, 1))
            if groups_local:
                offs = self._scan(ngroups)
                if ctx.get('blk') is not None:
                    sdp.sdp_part_compact_blocks(ptr(ctx['out_key']), ptr(ctx['out_cnt']), ctypes.byref(ctx['blk']),
                                                ptr(ngroups), ptr(offs), nfinal, ptr(keys), ptr(counts), s)
                else:
                    sdp.sdp_part_compact(ptr(ctx['out_key']), ptr(ctx['out_cnt']), ptr(starts), ptr(ngroups),
                                         ptr(offs), nfinal, ptr(keys), ptr(counts), s)
            extra_k, extra_c = [], []
            if hv:
                hh = hv['h_host']
                meta = hv['meta_host'] if isb else None
                for i in heavy_sel:
                    if isb:
                        extra_k.append(((hh[i] >> 40) << 40) | (meta[i] & ((1 << 40) - 1)))
                    else:
                        extra_k.append(inv_mix64(hh[i]))
                    extra_c.append(hc[i])
            if special:
                extra_k.append(inv_mix64(U64))
                extra_c.append(special)
            if extra_k:
                m = len(extra_k)
                keys[groups_local:groups_local + m] = to_dev(np.array(extra_k, dtype=np.uint64).view(np.int64),
                                                            torch.int64, self.device)
                counts[groups_local:groups_local + m] = to_dev(extra_c, torch.int64, self.device)
            tab.update({'slots': keys, 'counts': counts, 'capacity': max(total, 1)})
        return tab

    BITS32_DTYPES = (nat.I8, nat.I16, nat.I32, nat.I64, nat.U8, nat.U16, nat.U32, nat.U64)

    def _bits32_ok(self, col, bd):
        """The 32-bit partition + LDS bitmap distinct count (sdp_distinct32)
        applies: float32 keys, or an integral range < 2^32; and no heavy key in
        the pass-1 sample (a key with a large share of the rows would fill one
        final bucket)."""
        if not BITS32 or col.kind != 'fixed':
            return False
        if col.dtype == nat.F32:
            pass
        elif col.dtype in self.BITS32_DTYPES and bd is not None and bd[1] - bd[0] < (1 << 32):
            pass
        else:
            return False
        pre = self._heavy_pre or {}
        return pre.get(id(col)) is None

    def distinct_paths(self, cols, hints, bounds):
        """'bitmap' | 'bits32' | 'group' | 'table' per column: the path choice
        of describe._distinct_count / distinct_fixed on a single rank."""
        out = []
        for col, hint, bd in zip(cols, hints, bounds):
            if (bd is not None and col.kind == 'fixed' and col.dtype in self.BITMAP_DTYPES
                    and bd[1] - bd[0] + 1 <= nat.BITMAP_MAX_BITS):
                out.append('bitmap')
            elif hint * 4 > max(col.length, 1) and col.length >= (1 << 16):
                out.append('bits32' if self._bits32_ok(col, bd) else 'group')
            else:
                out.append('table')
        # wide tables of short columns (512 x 1e7): the
        # partitioning path fuses same-geometry columns into a few launches
        # (_group_middle_fused), where one sdp_distinct32 per column would pay
        # five launches and a host call each
        short32 = [i for i, p in enumerate(out) if p == 'bits32' and cols[i].length <= self.FUSE_MAX_RECS]
        if len(short32) >= self.FUSE_MIN_COLS:
            for i in short32:
                out[i] = 'group'
        return out

    def _distinct32_launch(self, col, lo):
        """sdp_distinct32 of `col` queued; returns the [distinct, rows] device
        pair.  When pass 2 took the level-1 count (numeric_stats_batch's
        count32_cols), the column is read once here instead of twice."""
        pre = self._counted.pop(id(col), None)
        h1 = None
        if pre is not None and pre.get('d32'):              # (a partitioning-path count is dropped)
            h1, out = pre['h1'], pre['stats']
        else:
            out = self._u64(2, zero=True)
        work = self._bytes(sdp.sdp_distinct32_workspace_bytes(col.length))
        cs = col.sdp()
        nat.annotate(_label(col, 'distinct32'), col_read_bytes(col) * (1 if h1 is not None else 2) + 4 * 5 * col.length)
        sdp.sdp_distinct32(ctypes.byref(cs), int(lo), ptr(h1), ptr(work), work.numel(), ptr(out), self._s())
        return out

    def distinct_batch(self, cols, hints, bounds, known=None, paths=None):
        """countDistinct of several NUM/DATE columns (describe.py:143) with
        the path choice of describe._distinct_count / distinct_fixed per column
        and the host readbacks shared: LDS bitmaps for small integral ranges
        (one readback for all), hash partitioning for the rest (group_batch).
        `bounds[i]` = (imin, imax) for integral columns with values, else None.
        `paths`: the caller's distinct_paths of these columns, taken before
        pass 2 consumed the heavy-key samples the choice reads (describe()
        passes them, so pass 2's pre-counts and this batch agree); computed
        here when absent.  Single rank only; returns [distinct count]."""
        out = list(known) if known is not None else [None] * len(cols)     # sorted columns: counted
        if paths is None:
            paths = self.distinct_paths(cols, hints, bounds)
        bm = [i for i, pth in enumerate(paths) if pth == 'bitmap' and out[i] is None]
        b32 = [i for i, pth in enumerate(paths) if pth == 'bits32' and out[i] is None]
        grp = [i for i, pth in enumerate(paths) if pth == 'group' and out[i] is None]
        if bm or b32:
            # bitmaps and 32-bit partitions queue without a host round trip: one
            # readback of every such column's count
            outs = [self._distinct_bitmap_launch(cols[i], bounds[i][0], bounds[i][1] - bounds[i][0] + 1) for i in bm]
            outs += [self._distinct32_launch(cols[i], bounds[i][0] if bounds[i] is not None else 0)[:1] for i in b32]
            for i in b32:                             # (their heavy-key samples go unused)
                (self._heavy_pre or {}).pop(id(cols[i]), None)
            for i, v in zip(bm + b32, self._host_u64(torch.cat(outs))):
                out[i] = int(v)
        if grp:
            for i, tab in zip(grp, self.group_batch([cols[i] for i in grp])):
                if tab is not None:
                    out[i] = tab['groups']
        for i, col in enumerate(cols):                  # global-table path / fallbacks
            if out[i] is None:
                out[i] = self.distinct_fixed(col, with_counts=False, capacity_hint=hints[i])['groups']
        return out

    def group_sharded(self, col):
        """group_sharded_batch of one column."""
        return self.group_sharded_batch([col])[0]

    def group_sharded_batch(self, cols, n_all=None):
        """countDistinct (describe.py:143) of fixed-width columns of a
        row-sharded table, on the partitioning kernels: level-1 buckets (top
        B1 hash bits) are owned by contiguous rank ranges, so after the local
        bucket scatter ONE all-to-all of 8-byte records hands every owner all
        records of its buckets; level 2 and the LDS de-duplication then run on
        the owner, and the group counts are all-reduced.  Heavy keys come from
        the pooled samples of all ranks (the same set everywhere) and are
        counted locally and all-reduced.  The columns share their host round
        trips and small collectives: ONE readback of every column's level-1
        bucket starts, ONE all-gather of every column's bucket sizes (which
        also give every rank its receive counts, so each all-to-all needs no
        count exchange), ONE all-reduce + readback of every column's group
        statistics.  Entries are None where the owner tables overflow (the
        caller takes the table-exchange path)."""
        comm, world, rank = self.comm, self.comm.world, self.comm.rank
        if not cols:
            return []
        s = self._s()
        B1 = self.SHARDED_B1
        nb1 = 1 << B1
        if n_all is None:                                 # (the caller usually knows the table's rows)
            n_all = int(comm.allreduce_sum(torch.full((1,), cols[0].length, dtype=torch.int64,
                                                         device=self.device)).item())
        target = sdp.sdp_part_bucket_target(0, 0)
        b2 = min(10, max(1, math.ceil(math.log2(max(2.0, n_all / nb1 / target)))))
        nb2 = 1 << b2
        lo = [(r * nb1) // world for r in range(world + 1)]
        ctxs = []
        for col in cols:                                  # level 1 counts of every column, no readback
            ctx = self._counted.pop(id(col), None)        # counted by pass 2 (sdp_pass2_count)
            if ctx is not None and (ctx.get('d32') or not ctx.get('sharded')):
                ctx = None                                # another path's count: recount
            if ctx is None:
                ctx = self._group_prepare_sharded(col)
                if ctx['n']:
                    nat.annotate(_label(col, 'count'), ctx['rb'])
                    sdp.sdp_part_rows(ctypes.byref(ctx['cs']), None, ctx['hvref'], B1, 0, ptr(ctx['h1']), None,
                                      None, ptr(ctx['hcnt']), ptr(ctx['stats']), s)
            grid = ctx['grid']
            ctx['o1'] = self._scan(ctx.pop('h1'))
            ctx['bsn_dev'] = torch.cat([ctx['o1'][0:nb1 * grid:grid], ctx['o1'][-1:]])
            ctxs.append(ctx)
        # every rank's level-1 bucket sizes in one all-gather and ONE readback
        # (the local bucket starts are the prefix sums of this rank's row; the
        # exclusive scan starts at 0)
        sizes = torch.cat([c['bsn_dev'][1:] - c['bsn_dev'][:-1] for c in ctxs])
        all_sizes = torch.stack(comm.allgather(sizes)).cpu().numpy().astype(np.int64).reshape(world, len(ctxs), nb1)
        bss = [np.concatenate([[0], np.cumsum(all_sizes[rank, i])]).astype(np.int64) for i in range(len(ctxs))]
        my0, my1 = lo[rank], lo[rank + 1]
        nmy = my1 - my0

        def owner_stage(ci, ctx, recv, S, part_tot):
            """Level 2 + LDS de-duplication of the records this rank owns."""
            col, stats = ctx['col'], ctx['stats']
            nrecv = int(recv.numel())
            if not nrecv:
                return
            # received layout: source-rank-major, my buckets in order inside each
            # part; chunks of <= PART_CHUNK records, ordered (bucket, source, chunk)
            part_base = np.concatenate([[0], np.cumsum(part_tot)[:-1]]).astype(np.int64)
            st0 = part_base[:, None] + np.concatenate([np.zeros((world, 1), np.int64),
                                                      np.cumsum(S, axis=1)[:, :-1]], axis=1)
            rin = nat.SdpRecords(recv.data_ptr(), None, None)
            if self._l2b_ok(False, b2, bool(ctx['hv'] and ctx['hv']['n'])):
                # level 2 into blocks: bucket bi = one segment per source rank
                lo_s = st0.T.reshape(-1)
                nat.annotate('u64/l2blocks', 2 * nrecv * 8)
                rf, keepf, blk, blk_keep = self._l2_blocks(rin, False, B1, b2, lo_s, lo_s + S.T.reshape(-1),
                                                           np.repeat(np.arange(nmy), world), nmy)
                ngroups = torch.zeros(nmy * nb2, dtype=torch.int32, device=self.device)
                nat.annotate('u64', nrecv * 8)
                sdp.sdp_part_dedup_blocks(ctypes.byref(rf), 0, None, ctypes.byref(blk), nmy * nb2,
                                          4 if id(col) in self._near_unique else 0, None, None, ptr(ngroups),
                                          ptr(stats), s)
                del keepf, rf, blk_keep
                return
            cnt = -(-S // PART_CHUNK)                                   # chunks per (source, bucket)
            cb, csrc = cnt.T.reshape(-1), np.tile(np.arange(world), nmy)
            bi_of = np.repeat(np.arange(nmy), world)
            rep_b, rep_src = np.repeat(bi_of, cb), np.repeat(csrc, cb)
            first = np.concatenate([[0], np.cumsum(cb)[:-1]])
            jj = np.arange(int(cb.sum()), dtype=np.int64) - np.repeat(first, cb)
            seg_start = st0[rep_src, rep_b] + jj * PART_CHUNK
            seg_end = np.minimum(st0[rep_src, rep_b] + S[rep_src, rep_b], seg_start + PART_CHUNK)
            nch = np.bincount(rep_b, minlength=nmy).astype(np.int64)
            k0 = np.concatenate([[0], np.cumsum(nch)[:-1]]).astype(np.int64)
            K = int(nch.sum())
            j = np.arange(K, dtype=np.int64) - k0[rep_b]
            ch = np.empty((K, 4), dtype=np.int64)
            ch[:, 0], ch[:, 1] = seg_start, seg_end
            ch[:, 2] = nb2 * k0[rep_b] + j
            ch[:, 3] = nch[rep_b]
            chunks = self._h2d(ch)
            h2 = torch.empty(nb2 * K, dtype=torch.int32, device=self.device)
            nat.annotate('u64/count', nrecv * 8)
            sdp.sdp_part_recs(ctypes.byref(rin), 0, ptr(chunks), K, B1, b2, 0, ptr(h2), None, None, s)
            o2 = self._scan(h2)
            rf, keepf = self._records(nrecv, False)
            nat.annotate('u64/scatter', 2 * nrecv * 8)
            sdp.sdp_part_recs(ctypes.byref(rin), 0, ptr(chunks), K, B1, b2, 1, None, ptr(o2),
                              ctypes.byref(rf), s)
            del h2
            sidx = (nb2 * k0[:, None] + np.arange(nb2)[None, :] * nch[:, None]).reshape(-1)
            sidx = np.append(sidx, nb2 * K)
            starts = o2[self._h2d(sidx)].contiguous()
            ngroups = torch.zeros(nmy * nb2, dtype=torch.int32, device=self.device)
            nat.annotate('u64', nrecv * 8)
            sdp.sdp_part_dedup(ctypes.byref(rf), 0, None, ptr(starts), nmy * nb2,
                               4 if id(col) in self._near_unique else 0, None, None, ptr(ngroups),
                               ptr(stats), s)
            del keepf, rf

        # pipelined: column i's all-to-all runs on the collective stream while
        # column i-1's owner stage runs on the compute stream (every rank
        # issues the exchanges in column order)
        pending = None
        for ci, (ctx, bs) in enumerate(zip(ctxs, bss)):
            col, stats = ctx['col'], ctx['stats']
            nrec = int(bs[-1])
            r1, keep1 = self._records(nrec, False)
            if nrec:
                nat.annotate(_label(col, 'scatter'), ctx['rb'] + nrec * 8)
                sdp.sdp_part_rows(ctypes.byref(ctx['cs']), None, ctx['hvref'], B1, 1, None, ptr(ctx['o1']),
                                  ctypes.byref(r1), ptr(ctx['hcnt']), ptr(stats), s)
            del ctx['o1'], ctx['bsn_dev']
            send = [int(bs[lo[r + 1]] - bs[lo[r]]) for r in range(world)]
            S = all_sizes[:, ci, my0:my1]                                   # [world, nmy]
            part_tot = S.sum(axis=1)
            recv, work = comm.alltoallv_known_async(keep1[0][:nrec], send, [int(x) for x in part_tot])
            if pending is not None:
                p_ci, p_ctx, p_recv, p_work, p_S, p_tot, p_keep = pending
                p_work.wait()
                del p_keep                     # the send buffer outlives its collective
                owner_stage(p_ci, p_ctx, p_recv, p_S, p_tot)
            pending = (ci, ctx, recv, work, S, part_tot, (keep1, r1))
            del keep1, r1
        if pending is not None:
            p_ci, p_ctx, p_recv, p_work, p_S, p_tot, p_keep = pending
            p_work.wait()
            del p_keep
            owner_stage(p_ci, p_ctx, p_recv, p_S, p_tot)
            pending = None
        # every column's group statistics in one all-reduce and one readback
        parts, spans = [], []
        for ctx in ctxs:
            st = ctx['stats'].clone()
            st[4] = st[4:68].sum()
            hv = ctx['hv']
            h = ctx['hcnt'][:max(hv['n'], 1)] if hv else ctx['hcnt'][:1]
            spans.append((sum(p.numel() for p in parts), h.numel()))
            parts += [st[:5], h]
        t = self._host_u64(comm.allreduce_sum(torch.cat(parts)))
        out = []
        for ctx, (o, hn) in zip(ctxs, spans):
            tt = t[o:o + 5 + hn]
            if tt[2] or tt[3]:
                out.append(None)
                continue
            hv = ctx['hv']
            heavy_present = sum(1 for c in tt[5:5 + (hv['n'] if hv else 0)] if c)
            groups = tt[4] + heavy_present + (1 if tt[1] else 0)
            out.append({'bytes': False, 'dense': False, 'rows': tt[0], 'max_key_rows': 0, 'col': ctx['col'],
                        'groups': groups, 'groups_local': groups, 'sharded': True})
        return out

    SHARDED_B1 = 10            # level-1 hash bits of the sharded grouping (buckets owned by rank ranges)

    def _group_prepare_sharded(self, col):
        """Level-1 geometry and buffers of group_sharded_batch for one column
        (the same as the single-rank count's, so sdp_pass2_count can fill it);
        heavy keys from the samples pooled over every rank."""
        n = col.length
        hv = self._heavy_keys(col, False, gather=True)
        rpb = sdp.sdp_part_rows_per_block(max(n, 1), 0)
        grid = max(1, -(-n // rpb))
        nb1 = 1 << self.SHARDED_B1
        ctx = {'col': col, 'n': n, 'cs': col.sdp(), 'hv': hv, 'stats': self._u64(68, zero=True),
               'hcnt': self._u64(max(hv['n'] if hv else 1, 1), zero=True), 'rb': col_read_bytes(col),
               'b1': self.SHARDED_B1, 'grid': grid, 'sharded': True,
               'h1': torch.zeros(nb1 * grid, dtype=torch.int32, device=self.device)}
        ctx['hvref'] = ctypes.byref(hv['struct']) if hv else None
        return ctx

    def distinct_paths_sharded(self, cols, hints, bounds, n_all):
        """'bitmap' | 'table' | 'group' per column: distinct_batch_sharded's
        path choice (identical on every rank: it reads merged pass-1 values
        and the global row count only)."""
        out = []
        for col, hint, bd in zip(cols, hints, bounds):
            if (bd is not None and col.kind == 'fixed' and col.dtype in self.BITMAP_DTYPES
                    and bd[1] - bd[0] + 1 <= nat.BITMAP_MAX_BITS):
                out.append('bitmap')
            elif hint is not None and hint * 4 <= max(n_all, 1):
                out.append('table')
            else:
                out.append('group')
        return out

    def distinct_batch_sharded(self, cols, hints, bounds, known=None, n_all=None, paths=None):
        """distinct_batch on a row-sharded table (every rank calls it with the
        same columns; hints/bounds come from the merged pass 1): bitmaps for
        small integral ranges, the global-table exchange for small key ranges,
        group_sharded_batch for the rest (shared round trips)."""
        comm = self.comm
        if n_all is None:                                 # (describe() passes the table's global rows)
            n_all = int(comm.allreduce_sum(torch.full((1,), cols[0].length if cols else 0, dtype=torch.int64,
                                                        device=self.device)).item()) if cols else 0
        out = list(known) if known is not None else [None] * len(cols)     # sorted columns: counted
        grp, bitmaps = [], []
        if paths is None:
            paths = self.distinct_paths_sharded(cols, hints, bounds, n_all)
        for i, (col, pth) in enumerate(zip(cols, paths)):
            bd = bounds[i]
            if out[i] is not None:
                continue
            if pth == 'bitmap':
                bitmaps.append((i, self._distinct_bitmap_dev(col, bd[0], bd[1] - bd[0] + 1)))
            elif pth == 'table':
                out[i] = self._distinct_fixed_table(col, False, hints[i])['groups']
            else:
                grp.append(i)
        for i, tab in zip(grp, self.group_sharded_batch([cols[i] for i in grp], n_all=n_all)):
            out[i] = tab['groups'] if tab is not None else \
                self._distinct_fixed_table(cols[i], False, hints[i])['groups']
        if bitmaps:                                       # every bitmap count in one readback
            for (i, _), v in zip(bitmaps, self._host_u64(torch.cat([d for _, d in bitmaps]))):
                out[i] = v
        return out

    def _scan(self, counts_i32):
        """Exclusive scan of int32 counts -> int64 offsets (n + 1 entries)."""
        n = counts_i32.numel()
        out = self._u64(n + 1)
        work = self._bytes(sdp.sdp_scan_workspace_bytes(n))
        sdp.sdp_scan_u32(ptr(counts_i32), n, ptr(out), ptr(work), work.numel(), self._s())
        return out

    BITMAP_DTYPES = (nat.I8, nat.I16, nat.I32, nat.I64, nat.U8, nat.U16, nat.U32)

    def _distinct_bitmap_launch(self, col, lo, range_, keep_bitmap=False):
        nw = (range_ + 31) // 32
        work = self._bytes(sdp.sdp_bitmap_workspace_bytes(col.length, range_))
        bm = torch.zeros(nw, dtype=torch.int32, device=self.device)      # (an empty shard writes nothing)
        out = self._u64(1, zero=True)
        cs = col.sdp()
        nat.annotate(_label(col), col_read_bytes(col))
        sdp.sdp_distinct_bitmap(ctypes.byref(cs), int(lo), int(range_), ptr(work), work.numel(), ptr(bm), ptr(out),
                                self._s())
        return (out, bm, nw) if keep_bitmap else out

    def distinct_bitmap(self, col, lo, range_):
        """countDistinct (describe.py:143) of an integral column whose values lie
        in [lo, lo + range_), range_ <= 2^20: LDS bitmaps (sdp_bitmap.hip).  Ranks
        all-gather their OR-ed bitmaps and re-reduce them."""
        return int(self._distinct_bitmap_dev(col, lo, range_).item())

    def _distinct_bitmap_dev(self, col, lo, range_):
        """distinct_bitmap's count as a one-element device tensor (no readback)."""
        out, bm, nw = self._distinct_bitmap_launch(col, lo, range_, keep_bitmap=True)
        if self.comm.sharded:
            allb = torch.cat(self.comm.allgather(bm))
            out.zero_()
            sdp.sdp_bitmap_reduce(ptr(allb), self.comm.world, nw, None, ptr(out), self._s())
        return out

    def distinct_fixed(self, col, with_counts=False, capacity_hint=None):
        """countDistinct over a fixed-width column (describe.py:143).

        Path choice (measured on MI355X at 1e9 rows, tools/bench_group.py):
        the radix-partitioned LDS grouping wins for near-unique keys (50 vs 80
        ms); a global table sized by a small key range (<= rows / 4) stays
        cache-resident and wins there (23 vs 44 ms)."""
        n = col.length
        if self.comm.sharded:         # the path choice must agree on every rank: decide on the global rows
            n = int(self.comm.allreduce_sum(torch.full((1,), n, dtype=torch.int64, device=self.device)).item())
        small_range = capacity_hint is not None and capacity_hint * 4 <= max(n, 1)
        if not self.comm.sharded and not small_range and col.length >= (1 << 16):
            tab = self.group(col, with_counts, dense=with_counts)
            if tab is not None:
                return tab
        if self.comm.sharded and not with_counts and not small_range:
            tab = self.group_sharded(col)          # collective: every rank takes this branch
            if tab is not None:
                return tab
        return self._distinct_fixed_table(col, with_counts, capacity_hint)

    def _distinct_fixed_table(self, col, with_counts=False, capacity_hint=None, row_counts=None, exchanged=False):
        """Global open-addressing table (fallback / small key ranges / multi-rank)."""
        bound = col.length if capacity_hint is None else min(capacity_hint, col.length)
        cap = _next_pow2(2 * max(bound, 1))
        slots, counts = self._table(cap, False, with_counts)
        stats = self._u64(4, zero=True)
        cs = col.sdp()
        nat.annotate(_label(col), col_read_bytes(col))
        sdp.sdp_hash_u64(ctypes.byref(cs), ptr(row_counts), ptr(slots), ptr(counts), cap, int(with_counts),
                         ptr(stats), self._s())
        st = self._host_u64(stats)
        groups = st[0] + (1 if st[2] else 0)
        tab = {'slots': slots, 'counts': counts, 'capacity': cap, 'bytes': False, 'max_key_rows': st[2],
               'rows': st[1], 'groups': groups, 'groups_local': st[0], 'col': col}
        if self.comm.sharded and not exchanged:
            tab = self._exchange_fixed(tab, with_counts)
        return tab

    def value_counts_bytes(self, col):
        """Groups of a byte column (describe.py:251).  The partitioning path
        aggregates the local rows (3-4x faster than the global table at 1.25e8
        rows: 7.4 vs 27 ms for 1e8 labels); on a sharded table its dense groups
        then go through the same owner exchange as the table path's."""
        if col.length >= (1 << 16):
            tab = self.group(col, True, dense=True)          # no collective inside
            if tab is not None:
                return self._exchange_bytes(tab) if self.comm.sharded else tab
        return self.value_counts_bytes_table(col)

    def value_counts_bytes_batch(self, cols):
        """value_counts_bytes of several byte columns with shared readbacks:
        ONE readback of every column's heavy-key sample, then per column the
        one-read records, the bucket-start readback and the scatters/dedup,
        and ONE readback of the group statistics of every column in flight
        (flushed under BYTES_BATCH_BYTES).  The grouping is local to the rank;
        on a sharded table each column's groups then take the owner exchange."""
        out = [None] * len(cols)
        big = [i for i, c in enumerate(cols) if c.length >= (1 << 16)]
        pre = self._heavy_bytes_pre
        if all(id(cols[i]) in pre for i in big):           # sampled with pass 1
            hvs = [pre.pop(id(cols[i])) for i in big]
        else:
            hvs = self._heavy_keys_batch([cols[i] for i in big])
        done = []

        def flush():
            # one readback of the group statistics of every column in flight;
            # the (key, count) outputs of each are compacted and then dropped
            if not done:
                return
            sizes = [ctx['stats_dev'].numel() for _, ctx in done]
            allst = self._host_u64(torch.cat([ctx['stats_dev'] for _, ctx in done]))
            off = 0
            for (i, ctx), m in zip(done, sizes):
                out[i] = self._group_end(ctx, allst[off:off + m], True)
                for key in ('out_key', 'out_cnt', 'starts', 'ngroups', 'stats_dev', 'blk', 'blk_keep'):
                    ctx.pop(key, None)
                off += m
            done.clear()

        held = 0
        counted = []

        def middles():
            # ONE readback of the level-1 bucket starts of every counted column
            if not counted:
                return
            flat = torch.cat([ctx['bsn_dev'] for _, ctx in counted]).cpu().numpy().astype(np.int64)
            off = 0
            for i, ctx in counted:
                m = ctx['bsn_dev'].numel()
                self._group_middle(ctx, flat[off:off + m])
                off += m
                done.append((i, ctx))
            counted.clear()

        for i, hv in zip(big, hvs):
            ctx = self._group_prepare(cols[i], True, hv=hv)
            if ctx is None:
                continue
            # a column in flight holds its one-read records (24 B per row) until
            # its middle stage, then 16 B per record of (key, count) outputs
            # until the shared statistics readback: both under a byte budget
            need = 40 * cols[i].length
            if (counted or done) and held + need > self.BYTES_BATCH_BYTES:
                middles()
                flush()
                held = 0
            self._group_count(ctx)
            self._group_scan(ctx)
            counted.append((i, ctx))
            held += need
        middles()
        flush()
        xch = []
        for i, c in enumerate(cols):
            # small columns, collisions, table overflow: the global table; when
            # sharded every column's local groups (either path: the choice is
            # rank-local) go through ONE batched owner exchange, in column order
            if out[i] is None:
                out[i] = self.value_counts_bytes_table(c, exchanged=True)
            if self.comm.sharded:
                xch.append(i)
        if xch:
            from .distributed import exchange_bytes_groups_batch
            for i, tab in zip(xch, exchange_bytes_groups_batch(self, [out[i] for i in xch])):
                out[i] = tab
        return out

    def value_counts_bytes_table(self, col, row_counts=None, exchanged=False, capacity=None):
        """Global open-addressing byte-key table (fallback / multi-rank path)."""
        pend = self.bytes_table_launch(col, row_counts, capacity)
        tab = self.bytes_table_finish(pend, self._host_u64(pend['stats']), col)
        if self.comm.sharded and not exchanged:
            tab = self._exchange_bytes(tab)
        return tab

    def bytes_table_launch(self, col, row_counts=None, capacity=None):
        """The global byte-key table of `col`, queued (no readback)."""
        cap = capacity if capacity is not None else _next_pow2(2 * max(col.length, 1))
        slots, counts = self._table(cap, True, True)
        stats = self._u64(4, zero=True)
        bc = col.sdp_bytes()
        nat.annotate(_label(col), col_read_bytes(col))
        sdp.sdp_hash_bytes(ctypes.byref(bc), ptr(row_counts), ptr(slots), ptr(counts), cap, ptr(stats), self._s())
        return {'slots': slots, 'counts': counts, 'capacity': cap, 'stats': stats}

    @staticmethod
    def bytes_table_finish(pend, st, col):
        """bytes_table_launch's tab from the host copy `st` of its statistics."""
        return {'slots': pend['slots'], 'counts': pend['counts'], 'capacity': pend['capacity'], 'bytes': True,
                'rows': st[1], 'groups': st[0], 'groups_local': st[0], 'col': col}

    # -- top-k by (count desc, key asc) ------------------------------------------
    def topk(self, tab, k=TOPK):
        """Returns [(slot, count)] of the k first groups; bytes keys compared
        bytewise, fixed keys by their order-preserving u64 value."""
        slots, counts, cap, isb = tab['slots'], tab['counts'], tab['capacity'], tab['bytes']
        flags = int(isb) | (2 if tab.get('dense') else 0)
        groups = tab['groups_local'] if 'groups_local' in tab else tab['groups']
        special = (not isb) and tab.get('max_key_rows', 0)
        bcol = tab['col'].sdp_bytes() if isb else None
        bref = ctypes.byref(bcol) if isb else None
        s = self._s()

        def select(cmin, cmax, limit):
            out = self._u64(max(limit, 1))
            on = self._u64(1, zero=True)
            sdp.sdp_table_select(ptr(slots), ptr(counts), cap, flags, cmin, cmax, ptr(out), ptr(on), limit, s)
            return out, on

        def sort_take(sel, n_dev, take):
            sdp.sdp_sort_groups(ptr(sel), ptr(n_dev), ptr(slots), ptr(counts), bref, s)
            # count, slot indices, counts and slot values in ONE readback
            # (indices past the count are masked to slot 0 before the gathers)
            t = max(1, min(take, sel.numel()))
            live = torch.arange(t, device=self.device) < n_dev[0]
            idx_d = torch.where(live, sel[:t], torch.zeros_like(sel[:t]))
            got = self._host_u64(torch.cat([n_dev[:1], idx_d, counts[idx_d], slots[idx_d]]))
            m = min(got[0], take)
            idx, cnt, val = got[1:1 + m], got[1 + t:1 + t + m], got[1 + 2 * t:1 + 2 * t + m]
            cache = tab.setdefault('_slotval', {})
            cache.update(zip(idx, val))
            return list(zip(idx, cnt))

        extra = []
        if special:                        # group of the key equal to EMPTY64 (kept outside the table)
            extra = [(None, special)]
        if groups <= k:
            sel, n_dev = select(1, U64, max(groups, 1))
            res = sort_take(sel, n_dev, k)
            return _merge_special(res, extra, k, tab)
        hist = self._u64(64, zero=True)
        sdp.sdp_table_count_log2_hist(ptr(slots), ptr(counts), cap, flags, ptr(hist), s)
        h = np.array(self._host_u64(hist), dtype=np.int64)
        cum = 0
        b = 63
        while b >= 0:
            cum += int(h[b])
            if cum >= k:
                break
            b -= 1
        b = max(b, 0)
        lo = 1 << b
        if cum <= GSORT_MAX:
            sel, n_dev = select(lo, U64, cum)
            return _merge_special(sort_take(sel, n_dev, k), extra, k, tab)
        # exact threshold T = k-th largest count inside [2^b, 2^(b+1))
        above = cum - int(h[b])
        need = k - above                      # rank from the top inside the bucket
        width = 1 << b
        while True:
            step = max(1, -(-width // 2048))
            ch = self._u64(2048, zero=True)
            sdp.sdp_table_count_hist(ptr(slots), ptr(counts), cap, flags, lo, step, ptr(ch), s)
            c = np.array(self._host_u64(ch), dtype=np.int64)
            nb = min(2048, -(-width // step))
            acc = 0
            j = nb - 1
            while j >= 0:
                if acc + int(c[j]) >= need:
                    break
                acc += int(c[j])
                j -= 1
            need -= acc
            if step == 1:
                T = lo + j
                n_eq = int(c[j])
                break
            lo = lo + j * step
            width = step
        gt_sel, gt_n = select(T + 1, U64, k)
        res = sort_take(gt_sel, gt_n, k)                    # < k groups, all in the top-k
        r_t = k - len(res)
        if n_eq <= GSORT_MAX:
            eq_sel, eq_n = select(T, T, n_eq)
            res += sort_take(eq_sel, eq_n, r_t)
        else:
            res += self._smallest_keys_among(select(T, T, n_eq), r_t, tab, sort_take)
        return _merge_special(res, extra, k, tab)

    def topk_batch(self, tabs, k=TOPK):
        """topk() of several tables with shared readbacks: ONE readback of the
        log2 count histograms of every table with more than k groups, ONE of
        every table's sorted top groups.  A table whose threshold bucket holds
        more than GSORT_MAX groups (heavy ties) takes topk() on its own."""
        s = self._s()
        out = [None] * len(tabs)
        info = []
        for tab in tabs:
            isb = tab['bytes']
            info.append({'flags': int(isb) | (2 if tab.get('dense') else 0),
                         'groups': tab['groups_local'] if 'groups_local' in tab else tab['groups'],
                         'bcol': tab['col'].sdp_bytes() if isb else None})
        hists = []
        for i, (tab, inf) in enumerate(zip(tabs, info)):
            if inf['groups'] > k:
                hist = self._u64(64, zero=True)
                sdp.sdp_table_count_log2_hist(ptr(tab['slots']), ptr(tab['counts']), tab['capacity'], inf['flags'],
                                              ptr(hist), s)
                hists.append((i, hist))
        hh = {}
        if hists:
            flat = np.array(self._host_u64(torch.cat([h for _, h in hists])), dtype=np.int64)
            hh = {i: flat[64 * j:64 * (j + 1)] for j, (i, _) in enumerate(hists)}
        pend = []
        for i, (tab, inf) in enumerate(zip(tabs, info)):
            slots, counts, cap = tab['slots'], tab['counts'], tab['capacity']
            if inf['groups'] <= k:
                cmin, limit = 1, max(inf['groups'], 1)
            else:
                h = hh[i]
                cum, b = 0, 63
                while b >= 0:
                    cum += int(h[b])
                    if cum >= k:
                        break
                    b -= 1
                b = max(b, 0)
                if cum > GSORT_MAX:
                    out[i] = self.topk(tab, k)
                    continue
                cmin, limit = 1 << b, cum
            sel = self._u64(max(limit, 1))
            on = self._u64(1, zero=True)
            sdp.sdp_table_select(ptr(slots), ptr(counts), cap, inf['flags'], cmin, U64, ptr(sel), ptr(on), limit, s)
            bref = ctypes.byref(inf['bcol']) if inf['bcol'] is not None else None
            sdp.sdp_sort_groups(ptr(sel), ptr(on), ptr(slots), ptr(counts), bref, s)
            t = max(1, min(k, sel.numel()))
            live = torch.arange(t, device=self.device) < on[0]
            idx_d = torch.where(live, sel[:t], torch.zeros_like(sel[:t]))
            pend.append((i, t, torch.cat([on[:1], idx_d, counts[idx_d], slots[idx_d]])))
        if pend:
            flat = self._host_u64(torch.cat([p for _, _, p in pend]))
            off = 0
            for i, t, p in pend:
                got = flat[off:off + p.numel()]
                off += p.numel()
                tab = tabs[i]
                m = min(got[0], k)
                idx, cnt, val = got[1:1 + m], got[1 + t:1 + t + m], got[1 + 2 * t:1 + 2 * t + m]
                tab.setdefault('_slotval', {}).update(zip(idx, val))
                special = (not tab['bytes']) and tab.get('max_key_rows', 0)
                out[i] = _merge_special(list(zip(idx, cnt)), [(None, special)] if special else [], k, tab)
        return out

    def global_topk_batch(self, items, k=TOPK):
        """global_topk of several (tab, col) pairs: the top groups of all tables
        with shared readbacks, then the byte values of all of them in two
        readbacks (bounds, bytes); each column's rank merge in column order."""
        tops = self.topk_batch([tab for tab, _ in items], k)
        byte_req = []
        values = [None] * len(items)
        for j, ((tab, col), top) in enumerate(zip(items, tops)):
            slots = [sl for sl, _ in top]
            if tab['bytes']:
                cache = tab.get('_slotval', {})
                rows = [(cache[sl] & ((1 << 40) - 1)) - 1 for sl in slots]
                byte_req.append((j, tab.get('src_col', col), rows, col))
            else:
                values[j] = self.group_values(tab, slots, col)
        for (j, _, _, _), vals in zip(byte_req, self.row_bytes_values_batch([r[1:] for r in byte_req])):
            values[j] = vals
        from .distributed import merge_topk_batch
        return merge_topk_batch(self.comm, [[(v, int(c)) for v, (_, c) in zip(vals, top)]
                                            for top, vals in zip(tops, values)], k)

    def _smallest_keys_among(self, sel_pack, r, tab, sort_take):
        """The r groups with the smallest keys among a large set of equal counts."""
        sel, n_dev = sel_pack
        n = int(n_dev.item())
        slots = tab['slots']
        if not tab['bytes']:
            keys = slots[sel[:n]].contiguous()
            kth = self.select_kth(keys, n_dev, r - 1, 0, EMPTY64)
            out = self._u64(r)
            on = self._u64(1, zero=True)
            sdp.sdp_select_by_value(ptr(sel), ptr(keys), ptr(n_dev), 0, kth, ptr(out), None, ptr(on), self._s())
            return sort_take(out, on, r)
        bcol = tab['col'].sdp_bytes()
        offset = 0
        need = r
        done = []
        while True:
            pre = self._u64(max(n, 1))
            sdp.sdp_group_prefix(ptr(sel), ptr(n_dev), ptr(slots), ctypes.byref(bcol), offset, ptr(pre), self._s())
            kth = self.select_kth(pre, n_dev, need - 1, 0, EMPTY64)
            below = self._u64(max(n, 1))
            bn = self._u64(1, zero=True)
            if kth > 0:
                sdp.sdp_select_by_value(ptr(sel), ptr(pre), ptr(n_dev), 0, kth - 1, ptr(below), None, ptr(bn),
                                        self._s())
            nb = int(bn.item())
            if nb:
                done += sort_take(below, bn, nb)
            need -= nb
            eq = self._u64(max(n, 1))
            en = self._u64(1, zero=True)
            sdp.sdp_select_by_value(ptr(sel), ptr(pre), ptr(n_dev), kth, kth, ptr(eq), None, ptr(en), self._s())
            ne = int(en.item())
            if ne <= GSORT_MAX:
                done += sort_take(eq, en, need)
                return done
            sel, n_dev, n = eq, en, ne
            offset += 8

    def global_topk(self, tab, col, k=TOPK):
        """[(value, count)] of the first k groups by (count desc, key asc) over
        every rank (each rank owns a hash partition of the groups)."""
        top = self.topk(tab, k)
        values = self.group_values(tab, [sl for sl, _ in top], col)
        pairs = [(v, int(c)) for v, (_, c) in zip(values, top)]
        from .distributed import merge_topk
        return merge_topk(self.comm, pairs, k)

    def group_values(self, tab, slot_list, col: DeviceColumn):
        """Host values of the groups at `slot_list` (None = the EMPTY64 key)."""
        cache = tab.get('_slotval', {})
        need = [sl for sl in slot_list if sl is not None and sl not in cache]
        if need:
            idx = to_dev(need, torch.int64, self.device)
            cache = dict(cache)
            cache.update(zip(need, self._host_u64(tab['slots'][idx])))
        if not tab['bytes']:
            return [fixed_key_to_value(EMPTY64 if sl is None else cache[sl], col) for sl in slot_list]
        src = tab.get('src_col', col)
        rows = [(cache[sl] & ((1 << 40) - 1)) - 1 for sl in slot_list]
        return self.row_bytes_values(src, rows, col)

    # -- first rows (limit(1) / limit(50)) ----------------------------------------
    def first_rows(self, col: DeviceColumn, k):
        """Values of the first k rows that survive na.drop, in row order."""
        if col.kind == 'null' or col.length == 0:
            from .distributed import merge_first_rows
            return merge_first_rows(self.comm, [], k)
        c = nat.SdpColumn()
        c.d_values = None
        c.d_validity = col.validity.data_ptr() if col.validity is not None else None
        c.validity_bit_offset = col.bit_offset
        c.length = col.length
        c.dtype = 0
        if col.kind == 'fixed':
            c = col.sdp()
        idx = self._u64(k)
        found = self._u64(1, zero=True)
        sdp.sdp_first_valid(ctypes.byref(c), k, ptr(idx), ptr(found), self._s())
        f = int(found.item())
        rows = [int(x) for x in idx[:f].cpu().tolist()]
        if col.kind == 'bytes':
            vals = self.row_bytes_values(col, rows, col)
        else:
            vals = self.fixed_row_values(col, rows)
        from .distributed import merge_first_rows
        return merge_first_rows(self.comm, vals, k)

    def fixed_row_values(self, col, rows):
        if not rows:
            return []
        if col.dtype == nat.BOOL:
            bits = []
            vb = col.values
            for r in rows:
                b = col.bit_offset + r
                bits.append(b)
            byts = vb[to_dev([b // 8 for b in bits], torch.int64, self.device)].cpu().tolist()
            return [bool((x >> (b % 8)) & 1) for x, b in zip(byts, bits)]
        tv = typed_values(col)
        v = tv[to_dev(rows, torch.int64, self.device)].cpu().numpy()
        if col.dtype == nat.U64:
            v = v.view(np.uint64)
        elif col.dtype == nat.U32:
            v = v.view(np.uint32)
        elif col.dtype == nat.U16:
            v = v.view(np.uint16)
        return [host_value(x, col) for x in v.tolist()]

    def row_bytes_values_batch(self, reqs):
        """row_bytes_values of several (src, rows, col) requests: ONE readback
        of every row's byte bounds, ONE of all their bytes."""
        out = [[] for _ in reqs]
        live = [(j, src, rows, col) for j, (src, rows, col) in enumerate(reqs) if rows]
        if not live:
            return out
        bounds = []
        for j, src, rows, col in live:
            # representative rows come from record metas the kernels wrote: one
            # outside the column means the records were not what the library
            # was told (sdp_part_dedup flags those as collisions); never gather it
            if min(rows) < 0 or max(rows) >= src.length:
                raise nat.NativeError('representative row %d outside the %d-row column %r (record layout '
                                      'mismatch?)' % (min(rows) if min(rows) < 0 else max(rows), src.length,
                                                      src.name))
            if src.fixed_width:
                w = src.fixed_width
                st = torch.tensor([r * w for r in rows], dtype=torch.int64)
                bounds.append(to_dev(torch.cat([st, st + w]), torch.int64, self.device))
            else:
                ri = to_dev(rows, torch.int64, self.device)
                o = src.offsets
                bounds.append(torch.cat([o[ri], o[ri + 1]]).to(torch.int64))
        se = torch.cat(bounds).cpu().tolist()                    # one readback of every bound
        off, gathers, spans = 0, [], []
        for (j, src, rows, col) in live:
            m = len(rows)
            starts, ends = se[off:off + m], se[off + m:off + 2 * m]
            off += 2 * m
            pos = np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in zip(starts, ends)])
            if pos.size:
                gathers.append(src.data[to_dev(pos, torch.int64, self.device)])
            spans.append((j, col, starts, ends, int(pos.size)))
        flat = torch.cat(gathers).cpu().numpy().tobytes() if gathers else b''   # one readback of all bytes
        p = 0
        for j, col, starts, ends, _ in spans:
            vals = []
            for a, b in zip(starts, ends):
                vals.append(bytes_value(flat[p:p + (b - a)], col))
                p += b - a
            out[j] = vals
        return out

    def row_bytes_values(self, src: DeviceColumn, rows, col: DeviceColumn):
        if not rows:
            return []
        if min(rows) < 0 or max(rows) >= src.length:        # (checked here, not by a device-side assert)
            raise nat.NativeError('row_bytes_values: a group row outside the column')
        if src.fixed_width:
            w = src.fixed_width
            starts = [r * w for r in rows]
            ends = [s + w for s in starts]
        else:
            ri = to_dev(rows, torch.int64, self.device)
            o = src.offsets
            se = torch.cat([o[ri], o[ri + 1]]).to(torch.int64).cpu().tolist()    # one readback
            starts, ends = se[:len(rows)], se[len(rows):]
        pos = np.concatenate([np.arange(a, b, dtype=np.int64) for a, b in zip(starts, ends)]) if rows else []
        flat = src.data[to_dev(pos, torch.int64, self.device)].cpu().numpy().tobytes() if len(pos) else b''
        out = []
        p = 0
        for a, b in zip(starts, ends):
            raw = flat[p:p + (b - a)]
            p += b - a
            out.append(bytes_value(raw, col))
        return out

    # ==========================================================================
    # Pearson (utils.py:20-36)
    # ==========================================================================
    def gram(self, cols: List[DeviceColumn], shifts, check_nan):
        n = cols[0].length
        C = len(cols)
        arr = (nat.SdpColumn * C)(*[c.sdp() for c in cols])
        cn = (ctypes.c_int32 * C)(*[int(x) for x in check_nan])
        work = self._bytes(sdp.sdp_gram_workspace_bytes(n, C))
        keep = torch.empty((n + 31) // 32 + 1, dtype=torch.int32, device=self.device)
        nat.annotate('', sum(n / 8.0 for c in cols if c.validity is not None))
        sdp.sdp_rowmask(arr, cn, C, ptr(work), work.numel(), ptr(keep), self._s())
        sh = self._h2d(np.array([float(x) for x in shifts], dtype=np.float64))   # (on self.stream, before sdp_gram)
        G = torch.empty(C * C, dtype=torch.float64, device=self.device)
        s = torch.empty(C, dtype=torch.float64, device=self.device)
        nn = torch.empty(1, dtype=torch.float64, device=self.device)
        nat.annotate('', sum(col_read_bytes(c) - (n / 8.0 if c.validity is not None else 0) for c in cols) + n / 8.0)
        sdp.sdp_gram(arr, C, ptr(keep), ptr(sh), ptr(work), work.numel(), ptr(G), ptr(s), ptr(nn), self._s())
        packed = self.comm.allreduce_sum(torch.cat([G, s, nn]))   # fp64 partial sums over ranks
        host = packed.cpu().numpy()
        return host[:C * C].reshape(C, C), host[C * C:C * C + C], float(host[-1])

    # ==========================================================================
    # multi-GPU exchanges (hash-partitioned groups)
    # ==========================================================================
    def _exchange_fixed(self, tab, with_counts):
        from .distributed import exchange_fixed_groups
        return exchange_fixed_groups(self, tab, with_counts)

    def _exchange_bytes(self, tab):
        from .distributed import exchange_bytes_groups
        return exchange_bytes_groups(self, tab)


def _merge_special(res, extra, k, tab):
    """Insert the side-counted EMPTY64 key group (largest key) into a sorted list."""
    if not extra:
        return res[:k]
    allg = res + extra
    allg.sort(key=lambda sc: (-sc[1], EMPTY64 if sc[0] is None else _slot_key_for_sort(tab, sc[0])))
    return allg[:k]


def _slot_key_for_sort(tab, slot):
    cached = tab.get('_slotval', {}).get(slot)
    return _u(cached) if cached is not None else _u(tab['slots'][slot].item())


SORTED_MIN_ROWS = 1 << 16      # single rank: smaller columns group quickly anyway


def merge_sorted_distinct(parts):
    """Rank-order merge of sdp_sorted_distinct outputs [distinct, violation,
    first key, last key] -> the column's distinct count, or None when it is not
    sorted (a rank saw a decrease, or a rank's first key is below the last key
    of the ranks before it).  Equal keys across a rank boundary are one value."""
    total, last = 0, None
    for d, viol, first, lastk in (tuple(int(v) for v in p) for p in parts):
        if viol:
            return None
        if d == 0:
            continue                                   # a rank with no valid rows
        total += d
        if last is not None:
            if first < last:
                return None
            if first == last:
                total -= 1
        last = lastk
    return total


def merge_pass1_results(parts):
    """Rank-order merge of sdp_pass1_result structs -> dict of plain numbers."""
    W = nat.MAX_WINDOWS
    out = {
        'count': sum(p.count for p in parts), 'n_valid': sum(p.n_valid for p in parts),
        'n_nan': sum(p.n_nan for p in parts), 'n_zero': sum(p.n_zero for p in parts),
        'imin': min(p.imin for p in parts), 'imax': max(p.imax for p in parts),
        'dmin': min(p.dmin for p in parts), 'dmax': max(p.dmax for p in parts),
        'shift': parts[0].shift,
        's1': math.fsum([x for p in parts for x in (p.s1_hi, p.s1_lo)]),
        's1_hi': 0.0, 's1_lo': 0.0,
        's2': math.fsum([p.s2 for p in parts]),
        's3': math.fsum([x for p in parts for x in (p.s3_hi, p.s3_lo)]),
        's4': math.fsum([p.s4 for p in parts]),
        'w_gt': [sum(p.w_gt[w] for p in parts) for w in range(W)],
        'w_eq_lo': [sum(p.w_eq_lo[w] for p in parts) for w in range(W)],
        'w_eq_hi': [sum(p.w_eq_hi[w] for p in parts) for w in range(W)],
        'w_in': [sum(p.w_in[w] for p in parts) for w in range(W)],
        'w_overflow': 0,
    }
    # s1 as an unevaluated pair (hi + lo) exact to ~2^-106 for the mean
    hi = math.fsum([x for p in parts for x in (p.s1_hi, p.s1_lo)])
    lo = float(sum((Fraction(x) for p in parts for x in (p.s1_hi, p.s1_lo)), Fraction(0)) - Fraction(hi))
    out['s1_hi'], out['s1_lo'] = hi, lo
    isum = 0
    for p in parts:
        isum = (isum + p.isum) & U64
    out['isum'] = isum - (1 << 64) if isum >= (1 << 63) else isum
    for p in parts:
        out['w_overflow'] |= p.w_overflow
    return out


def moments(p1, is_int):
    """Spark Average / Sum / CentralMomentAgg outputs from the
    shifted power sums about K."""
    n = p1['count']
    K = p1['shift']
    s1, s2, s3, s4 = p1['s1'], p1['s2'], p1['s3'], p1['s4']
    # Spark Average = (double sum) / count: the sum is rounded once, from the
    # exact K*n + s1 (Fraction arithmetic on the host, a handful of operations)
    dsum = float(Fraction(K) * n + Fraction(p1['s1_hi']) + Fraction(p1['s1_lo'])) if n else 0.0
    mean = dsum / n if n else float('nan')
    m = s1 / n if n else 0.0
    M2 = s2 - s1 * s1 / n if n else 0.0
    M3 = s3 - 3.0 * m * s2 + 2.0 * n * m ** 3
    M4 = s4 - 4.0 * m * s3 + 6.0 * m * m * s2 - 3.0 * n * m ** 4
    if M2 < 0:
        M2 = 0.0
    if n == 0:
        variance = std = skew = kurt = float('nan')
    else:
        variance = float('nan') if n == 1 else M2 / (n - 1.0)
        std = float('nan') if n == 1 else math.sqrt(variance)
        skew = float('nan') if M2 == 0 else math.sqrt(n) * M3 / math.sqrt(M2 * M2 * M2)
        kurt = float('nan') if M2 == 0 else n * M4 / (M2 * M2) - 3.0
    if is_int:
        mn, mx, total = float(p1['imin']), float(p1['imax']), float(p1['isum'])
    else:
        mn, mx, total = p1['dmin'], p1['dmax'], dsum
    return {'min': mn, 'max': mx, 'sum': total, 'mean': mean, 'variance': variance, 'std': std,
            'skewness': skew, 'kurtosis': kurt}


# ----------------------------------------------------------------------------
# key / value conversions for host assembly
# ----------------------------------------------------------------------------

_TORCH_DT = {nat.I8: torch.int8, nat.I16: torch.int16, nat.I32: torch.int32, nat.I64: torch.int64,
             nat.U8: torch.uint8, nat.U16: torch.int16, nat.U32: torch.int32, nat.U64: torch.int64,
             nat.F32: torch.float32, nat.F64: torch.float64}


def typed_values(col: DeviceColumn):
    """The column's value bytes viewed as its element type (length rows)."""
    t = _TORCH_DT[col.dtype]
    es = nat.ELEM_SIZE[col.dtype]
    v = col.values
    if v.dtype == torch.uint8:
        v = v[:col.length * es].view(t)
    return v[:col.length]


def host_value(x, col: DeviceColumn):
    """A raw element as the driver sees it after toPandas (numpy scalar)."""
    st = col.spark_type
    if st == 'date':
        import datetime
        return datetime.date(1970, 1, 1) + datetime.timedelta(days=int(x))
    if st == 'timestamp':
        import pandas as pd
        return pd.Timestamp(int(x), unit=col.ts_unit)
    if col.dtype in (nat.F32, nat.F64):
        return np.float64(x)
    if col.dtype == nat.U64:
        import decimal
        return decimal.Decimal(int(x))
    return np.int64(x)


def fixed_key_to_value(k, col: DeviceColumn):
    if col.dtype == nat.BOOL:
        return bool(k)
    if col.dtype in (nat.U8, nat.U16, nat.U32):
        return np.int64(k)
    if col.dtype == nat.U64:
        import decimal
        return decimal.Decimal(int(k))
    if col.dtype in (nat.F32, nat.F64):
        return np.float64(key_to_float(k))
    return host_value(key_to_int(k), col)


def bytes_value(raw: bytes, col: DeviceColumn):
    if col.spark_type == 'string':
        return raw.decode('utf-8', errors='replace')
    if col.spark_type.startswith('decimal'):
        return decimal_from_key(raw, col.decimal_scale)
    return bytes(raw)
