"""sdp_value_counts_topk (the coarse C-ABI entry for describe.py:251-263) on
the paths the C host's 5000-label column never reaches, called through ctypes
with device buffers (the same entry the C host binds):

* a zipf string column whose heavy-key sample holds more than 256 keys (the
  records kernel takes up to SDP_HEAVY_MAX_REC = 1024 of them);
* more than SDP_GSORT_MAX groups tied at the k-th count, for a fixed-width and
  a byte column (the smallest-keys cut; byte keys by 8-byte prefixes,
  recursively, since every key shares its first 8 bytes);
* more than SDP_GSORT_MAX groups in the top log2 count bucket, so the exact
  threshold is refined with a step > 1;
* k > SDP_GSORT_MAX is rejected.

Expected results: collections.Counter with (count desc, key asc).  Needs an MI355X."""

import ctypes
from collections import Counter

import numpy as np
import pyarrow as pa
import pytest

import datagen

pytestmark = pytest.mark.gpu


def _topk(arr, k):
    import torch
    from spark_df_profiling import _native as nat
    from spark_df_profiling._native import sdp, ptr
    from spark_df_profiling.columns import DeviceTable
    t = DeviceTable.from_arrow(pa.table({'c': arr}))
    col = t.columns[0]
    isb = col.kind == 'bytes'
    ws = sdp.sdp_value_counts_workspace_bytes(col.length, int(isb))
    work = torch.empty(ws, dtype=torch.uint8, device='cuda')
    res = nat.SdpTopkResult()
    top = (nat.SdpTopkEntry * max(k, 1))()
    cs = None if isb else col.sdp()
    bc = col.sdp_bytes() if isb else None
    sdp.sdp_value_counts_topk(ctypes.byref(cs) if cs is not None else None,
                              ctypes.byref(bc) if bc is not None else None, k, ptr(work), ws, ctypes.byref(res),
                              top, nat.stream_handle())
    return res, [(top[i].key, top[i].count) for i in range(res.n_top)]


def _want(values, k):
    c = Counter(values)
    return sorted(c.items(), key=lambda kv: (-kv[1], kv[0]))[:k], len(c)


def _distinct_ints(g, lo, hi, m):
    """m distinct int64 in [lo, hi), random order (no population array)."""
    u = np.unique(g.integers(lo, hi, 2 * m + 64, dtype=np.int64))
    assert u.size >= m
    return g.permutation(u)[:m]


def _i64_key(v):
    return (int(v) + (1 << 63)) & ((1 << 64) - 1)          # order-preserving u64 of an int64


def test_topk_more_than_256_heavy_string_keys():
    g = datagen.rng(31)
    n = 600_000
    lab = np.minimum(g.zipf(1.1, n), 100_000)
    vals = ['L%05x' % x for x in lab]
    # (the 65536-row heavy sample sees well over 256 labels >= 3 times)
    samp = Counter(vals[i] for i in np.linspace(0, n - 1, 65536).astype(np.int64))
    assert sum(1 for c in samp.values() if c >= 3) > 256
    res, got = _topk(pa.array(vals, type=pa.large_string()), 50)
    want, groups = _want(vals, 50)
    assert (res.groups, res.rows, res.path) == (groups, n, 1)
    assert [(vals[r], c) for r, c in got] == want


def test_topk_small_column_heavy_keys_capped_to_row_kernels():
    # a few thousand rows (b1 == 0: the row kernels, whose heavy tables hold
    # SDP_HEAVY_MAX keys) with 400 labels seen >= 3 times in the whole-column
    # sample: sdp_api.cpp's cap_to trims the heavy keys to 256, the rest
    # become partition records; groups, rows and top-k as Counter says
    g = datagen.rng(34)
    vals = ['H%03d' % i for i in range(400)] * 10 + ['s%d' % i for i in range(600)]
    vals = [vals[i] for i in g.permutation(len(vals))]
    assert sum(1 for c in Counter(vals).values() if c >= 3) > 256
    res, got = _topk(pa.array(vals, type=pa.large_string()), 50)
    want, groups = _want(vals, 50)
    assert (res.groups, res.rows) == (groups, len(vals))
    assert [(vals[r], c) for r, c in got] == want


def test_topk_fixed_ties_beyond_gsort_max():
    g = datagen.rng(32)
    tied = _distinct_ints(g, -10 ** 9, 10 ** 9, 20_000)
    top = _distinct_ints(g, 2 * 10 ** 9, 3 * 10 ** 9, 10)
    v = np.concatenate([np.repeat(tied, 2), np.repeat(top, 5), np.arange(4 * 10 ** 9, 4 * 10 ** 9 + 60_000)])
    g.shuffle(v)
    res, got = _topk(pa.array(v), 50)
    want, groups = _want(v.tolist(), 50)
    assert res.groups == groups and res.rows == v.size
    assert got == [(_i64_key(x), c) for x, c in want]


def test_topk_byte_ties_beyond_gsort_max_shared_prefix():
    g = datagen.rng(33)
    ids = g.permutation(20_000)
    vals = ['common-prefix/%08d' % i for i in np.repeat(ids, 2)] + ['zz%d' % i for i in range(30)] * 3 + \
           ['single-%d' % i for i in range(70_000)]
    order = g.permutation(len(vals))
    vals = [vals[i] for i in order]
    res, got = _topk(pa.array(vals, type=pa.large_string()), 50)
    want, groups = _want(vals, 50)
    assert res.groups == groups
    assert [(vals[r], c) for r, c in got] == want


def test_topk_threshold_refined_with_step():
    # 9000 groups with counts in [4096, 8096): the top log2 bucket holds more
    # than SDP_GSORT_MAX groups and is 4096 wide, so the threshold refinement
    # first runs with step 2
    g = datagen.rng(34)
    keys = _distinct_ints(g, 0, 2 ** 40, 9000)
    cnt = g.integers(4096, 8096, 9000)
    v = np.repeat(keys, cnt)
    g.shuffle(v)
    res, got = _topk(pa.array(v), 50)
    order = sorted(zip(keys.tolist(), cnt.tolist()), key=lambda kc: (-kc[1], kc[0]))[:50]
    assert res.groups == 9000 and res.rows == v.size
    assert got == [(_i64_key(x), c) for x, c in order]


def test_topk_k_above_gsort_max_rejected():
    from spark_df_profiling import _native as nat
    with pytest.raises(nat.NativeError, match='k = 8193'):
        _topk(pa.array(np.arange(100_000, dtype=np.int64)), 8193)
