"""The partitioned grouping path (sdp_part.hip) vs numpy / the oracle, on
columns large enough (>= 2^16 rows) to take it: heavy keys, skew, long and
empty strings, nulls, NaN / -0.0, and the two u64 keys the kernels treat
specially (UINT64_MAX, and the key whose hash is UINT64_MAX).  Needs an MI355X."""

import numpy as np
import pyarrow as pa
import pytest

import datagen
from compare import assert_describe_equal

pytestmark = pytest.mark.gpu

N = 300_007
SPECIAL = [0xFFFFFFFFFFFFFFFF, 0x74A6576574A65765]     # UINT64_MAX, inv_mix64(UINT64_MAX)


def _engine_groups(arr):
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.engine import Engine
    t = DeviceTable.from_arrow(pa.table({'c': arr}))
    e = Engine()
    col = t.columns[0]
    return e, col


def _u64_table_groups(tab):
    import torch
    k = tab['slots'][:tab['groups']].cpu().numpy().view(np.uint64)
    c = tab['counts'][:tab['groups']].cpu().numpy()
    o = np.argsort(k)
    return k[o], c[o]


@pytest.mark.parametrize('kind', ['uniform', 'skewed', 'special'])
def test_group_u64_counts_exact(kind):
    g = datagen.rng(99)
    if kind == 'uniform':
        v = g.integers(0, 2 ** 63, N, dtype=np.uint64)
    elif kind == 'skewed':
        v = np.minimum(g.zipf(1.1, N), 10 ** 7).astype(np.uint64)
    else:
        v = g.integers(0, 50_000, N, dtype=np.uint64)
        v[g.random(N) < 0.2] = np.uint64(SPECIAL[0])
        v[g.random(N) < 0.1] = np.uint64(SPECIAL[1])
    e, col = _engine_groups(pa.array(v, type=pa.uint64()))
    tab = e.group(col, with_counts=True)
    assert tab is not None
    keys, counts = _u64_table_groups(tab)
    want_k, want_c = np.unique(v, return_counts=True)
    assert tab['groups'] == len(want_k)
    assert tab['rows'] == N
    assert np.array_equal(keys, want_k)
    assert np.array_equal(counts, want_c)


@pytest.mark.parametrize('dtype', ['f64', 'f32', 'i32', 'i16'])
def test_group_distinct_only(dtype):
    g = datagen.rng(5)
    if dtype == 'f64':
        v = g.standard_normal(N)
        v[g.random(N) < 0.05] = np.nan
        v[g.random(N) < 0.05] = -0.0
        v[g.random(N) < 0.05] = 0.0
        v[g.random(N) < 0.3] = 2.5
        arr, want = pa.array(v, mask=g.random(N) < 0.1), None
    elif dtype == 'f32':
        v = g.random(N).astype(np.float32)
        arr = pa.array(v)
    elif dtype == 'i32':
        v = g.integers(-2 ** 31, 2 ** 31 - 1, N).astype(np.int32)
        arr = pa.array(v, mask=g.random(N) < 0.05)
    else:
        v = g.integers(-2 ** 15, 2 ** 15, N).astype(np.int16)
        arr = pa.array(v)
    e, col = _engine_groups(arr)
    tab = e.group(col, with_counts=False, dense=False)
    assert tab is not None
    vals = arr.to_numpy(zero_copy_only=False)
    valid = ~np.asarray(arr.is_null().to_numpy(zero_copy_only=False))
    x = np.asarray(vals)[valid]
    if x.dtype.kind == 'f':
        x = x.astype(np.float64)
        x[x == 0] = 0.0
        n_nan = int(np.isnan(x).any())
        want = len(np.unique(x[~np.isnan(x)])) + n_nan
    else:
        want = len(np.unique(x))
    assert tab['groups'] == want
    assert tab['rows'] == int(valid.sum())


def _strings():
    g = datagen.rng(17)
    base = ['', 'a', 'ab', 'Élysée', 'x' * 16, 'y' * 17, 'long-string-%s' % ('z' * 40)]
    tail = ['t%07d' % i for i in range(200_000)]
    longs = ['L%06d-%s' % (i, 'q' * (i % 30)) for i in range(5000)]
    pick = g.random(N)
    z = np.minimum(g.zipf(1.3, N), len(tail)) - 1
    out = np.empty(N, dtype=object)
    for i in range(N):
        p = pick[i]
        if p < 0.3:
            out[i] = base[int(p * 100) % len(base)]
        elif p < 0.8:
            out[i] = tail[z[i]]
        else:
            out[i] = longs[int(p * 1e6) % len(longs)]
    return out, g.random(N) < 0.05


@pytest.mark.parametrize('atype', [pa.string(), pa.large_string(), pa.binary()])
def test_group_bytes_counts_exact(atype):
    vals, mask = _strings()
    if atype == pa.binary():
        arr = pa.array([s.encode() for s in vals], type=atype, mask=mask)
    else:
        arr = pa.array(vals.tolist(), type=atype, mask=mask)
    e, col = _engine_groups(arr)
    tab = e.group(col, with_counts=True)
    assert tab is not None
    m = tab['groups']
    slots = tab['slots'][:m].cpu().numpy().view(np.uint64)
    counts = tab['counts'][:m].cpu().numpy()
    rows = [(int(s) & ((1 << 40) - 1)) - 1 for s in slots]
    got_vals = e.row_bytes_values(col, rows, col)
    got = dict(zip(got_vals, counts.tolist()))
    assert len(got) == m                          # every group a different value
    from collections import Counter
    want = Counter(v for v, nul in zip(vals, mask) if not nul)
    if atype == pa.binary():
        want = Counter({k.encode(): c for k, c in want.items()})
    assert got == dict(want)
    assert tab['rows'] == int((~mask).sum())


def test_describe_large_categorical():
    """The categorical table above the partition threshold, through describe()."""
    import oracle
    from spark_df_profiling import describe
    t = datagen.categorical_table(N, seed=21)
    got = describe(t, plots=False)
    want, _ = oracle.profile_raw(t)
    assert_describe_equal(got, want)


def _dedup_buckets(buckets, flags):
    """sdp_part_dedup (distinct only) over hand-made final buckets of u64 hashes."""
    import ctypes
    import torch
    from spark_df_profiling import _native as nat
    from spark_df_profiling._native import sdp, ptr
    h = np.concatenate(buckets).astype(np.uint64)
    starts = np.concatenate([[0], np.cumsum([len(b) for b in buckets])]).astype(np.int64)
    dev = torch.device('cuda', 0)
    d_h = torch.from_numpy(h.view(np.int64)).to(dev)
    d_s = torch.from_numpy(starts).to(dev)
    stats = torch.zeros(68, dtype=torch.int64, device=dev)
    rin = nat.SdpRecords(d_h.data_ptr(), None, None)
    rc = sdp.sdp_part_dedup(ctypes.byref(rin), 0, None, ptr(d_s), len(buckets), flags, None, None, None, ptr(stats),
                            nat.stream_handle())
    assert rc == 0
    st = stats.cpu().numpy()
    return int(st[4:68].sum()), int(st[3])


@pytest.mark.parametrize('direct', [0, 4])
def test_wave_dedup_kernels(direct):
    """The wave dedup kernels (read-first 2048-slot tables; near-unique
    mode: the half-space tables) on crafted final buckets: single and
    multi-batch buckets, duplicates, keys sharing one home slot (collision list
    and its overflow), buckets around one 1024-record batch, empty buckets."""
    g = datagen.rng(7)
    b = []
    for _ in range(300):                                   # ordinary buckets with repeats
        m = int(g.integers(0, 1200))
        u = g.integers(0, 2 ** 63, max(1, m // 2), dtype=np.uint64)
        b.append(u[g.integers(0, len(u), m)] if m else np.zeros(0, np.uint64))
    same_home = (g.integers(0, 2 ** 52, 900, dtype=np.uint64) << np.uint64(11)) | np.uint64(77)
    b.append(np.repeat(same_home[:300], 2))                # 300 keys, one home slot
    b.append(same_home)                                    # 900 keys, one home: list overflow
    big = g.integers(0, 2 ** 63, 1500, dtype=np.uint64)
    b.append(big[g.integers(0, 1500, 6000)])               # multi-batch bucket (probe limit path)
    b.append(np.zeros(0, np.uint64))
    u = g.integers(0, 2 ** 63, 1281, dtype=np.uint64)
    b.append(u[:1024])                                     # one whole batch, all distinct
    b.append(u[:1025])                                     # one past it: two batches
    b.append(u)
    b.append(u[g.integers(0, 40, 1280)])                   # 40 keys repeated
    b.append(np.full(1, 12345, np.uint64))
    groups, full = _dedup_buckets(b, direct)
    want = sum(len(np.unique(x)) for x in b)
    assert full == 0
    assert groups == want


def _distinct32(arr, lo=0):
    import torch
    from spark_df_profiling import _native as nat
    from spark_df_profiling._native import sdp, ptr
    e, col = _engine_groups(arr)
    out = torch.zeros(2, dtype=torch.int64, device='cuda')
    work = torch.empty(sdp.sdp_distinct32_workspace_bytes(col.length), dtype=torch.uint8, device='cuda')
    cs = col.sdp()
    import ctypes
    sdp.sdp_distinct32(ctypes.byref(cs), int(lo), None, ptr(work), work.numel(), ptr(out), nat.stream_handle(None))
    torch.cuda.synchronize()
    d, rows = [int(x) for x in out.cpu()]
    return d, rows


@pytest.mark.parametrize('case', ['f32_norm', 'f32_special', 'i32_full', 'u32_full', 'i64_window', 'tiny', 'f32_groups'])
def test_distinct32_exact(case):
    """sdp_distinct32 (4-byte records in 64 x 64 buckets + LDS bitmaps) vs
    numpy, nulls skipped, NaN one value, -0.0 == 0.0, the ends of the 32-bit
    key space (describe.py:143); 'f32_groups' is long enough (> 2 x 64 x 65536
    rows) for the level-2 scatter to split each bucket's chunks over several
    workgroups."""
    g = datagen.rng(17)
    n = {'tiny': 1000, 'f32_groups': 9_000_017}.get(case, N)
    lo = 0
    mask = g.random(n) < 0.07
    if case in ('f32_norm', 'f32_groups'):
        v = g.standard_normal(n).astype(np.float32)
    elif case == 'f32_special':
        v = g.standard_normal(n).astype(np.float32)
        v[g.random(n) < 0.05] = np.nan
        v[g.random(n) < 0.02] = np.float32(np.nan) * -1
        v[g.random(n) < 0.03] = 0.0
        v[g.random(n) < 0.03] = -0.0
        v[:4] = [np.inf, -np.inf, np.finfo(np.float32).max, np.finfo(np.float32).tiny]
    elif case == 'i32_full':
        v = g.integers(-2 ** 31, 2 ** 31, n).astype(np.int32)
        v[:2] = [np.iinfo(np.int32).min, np.iinfo(np.int32).max]
        lo = int(v.min())
    elif case == 'u32_full':
        v = g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        v[:2] = [0, np.iinfo(np.uint32).max]
        lo = int(v.min())
    elif case == 'i64_window':
        v = (10 ** 12 + g.integers(0, 2 ** 32, n, dtype=np.int64)).astype(np.int64)
        v[:2] = [10 ** 12, 10 ** 12 + 2 ** 32 - 1]
        lo = int(v.min())
    else:
        v = g.integers(0, 300, n).astype(np.int32)
    mask[:2] = False
    d, rows = _distinct32(pa.array(v, mask=mask), lo)
    x = v[~mask]
    if x.dtype.kind == 'f':
        x = np.where(x == 0, np.float32(0), x)                     # -0.0 groups with 0.0
        want = len(np.unique(x[~np.isnan(x)])) + int(np.isnan(x).any())
    else:
        want = len(np.unique(x))
    assert (d, rows) == (want, int((~mask).sum()))


@pytest.mark.parametrize('copies', [1, 3])
def test_distinct32_describe_path(copies, monkeypatch):
    """describe() routes float32 and < 2^32-range integral columns without
    heavy keys to sdp_distinct32 and matches the oracle; with >= 8 numeric
    columns (the batched pass 2) their level-1 count rides pass 2's read."""
    import oracle
    from spark_df_profiling import describe
    from spark_df_profiling.engine import Engine
    g = datagen.rng(23)
    n = 200_003
    cols = {}
    for k in range(copies):
        cols['f32_%d' % k] = pa.array(g.standard_normal(n).astype(np.float32), mask=g.random(n) < 0.05)
        cols['i64_2p31_%d' % k] = pa.array(g.integers(-2 ** 31, 2 ** 31, n))
        cols['u32_%d' % k] = pa.array(g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32))
    t = pa.table(cols)
    # (9 short columns would otherwise take the fused wide-table partitioning)
    monkeypatch.setattr(Engine, 'FUSE_MIN_COLS', 100)
    seen, pre = [], []
    orig = Engine._distinct32_launch

    def spy(self, col, lo):
        seen.append(col.name)
        c = self._counted.get(id(col))
        pre.append(bool(c is not None and c.get('d32')))
        return orig(self, col, lo)
    Engine._distinct32_launch = spy
    try:
        assert_describe_equal(describe(t, plots=False), oracle.describe(t))
    finally:
        Engine._distinct32_launch = orig
    assert sorted(seen) == sorted(cols)
    assert all(pre) == (len(cols) >= 8) and (any(pre) == (len(cols) >= 8))


def test_wide_short_tables_keep_fused_partitioning():
    """>= 8 short (<= 2^26-row) 32-bit key columns keep the fused wide-table
    partitioning path (one launch per stage for all of them), not one
    sdp_distinct32 each (engine.distinct_paths)."""
    from spark_df_profiling.engine import Engine
    from spark_df_profiling.columns import DeviceTable
    g = datagen.rng(29)
    n = 100_000
    t = pa.table({'f%d' % k: pa.array(g.standard_normal(n).astype(np.float32)) for k in range(9)})
    dt = DeviceTable.from_arrow(t)
    e = Engine()
    paths = e.distinct_paths(dt.columns, [n] * 9, [None] * 9)
    assert paths == ['group'] * 9
    assert e.distinct_paths(dt.columns[:3], [n] * 3, [None] * 3) == ['bits32'] * 3


def test_byte_dedup_out_of_range_metas():
    """Byte records whose metas point outside the column (records that are not
    what the library was told, e.g. a layout mismatch between engine and
    library) are flagged as a collision by sdp_part_dedup -- never read -- and
    the exact recount on the global table gives the right groups."""
    import ctypes
    import torch
    from collections import Counter
    from spark_df_profiling import _native as nat
    from spark_df_profiling._native import sdp, ptr
    g = datagen.rng(11)
    base = ['k%03d' % i for i in range(300)] + ['a long string of more than sixteen bytes #%03d' % i
                                               for i in range(200)]
    vals = [base[i] for i in g.integers(0, len(base), 6000)]
    e, col = _engine_groups(pa.array(vals, type=pa.large_string()))
    bc = col.sdp_bytes()
    dev, s = e.device, nat.stream_handle()
    n = col.length
    rpb = sdp.sdp_part_rows_per_block(n, 1)
    grid = max(1, -(-n // rpb))
    h1 = torch.zeros(grid, dtype=torch.int32, device=dev)
    st0 = torch.zeros(68, dtype=torch.int64, device=dev)
    sdp.sdp_part_rows(None, ctypes.byref(bc), None, 0, 0, ptr(h1), None, None, None, ptr(st0), s)
    offs = e._scan(h1)
    nrec = int(offs[-1].item())
    assert nrec == n
    k0, k1, meta = (torch.empty(nrec, dtype=torch.int64, device=dev) for _ in range(3))
    rec = nat.SdpRecords(k0.data_ptr(), k1.data_ptr(), meta.data_ptr())
    sdp.sdp_part_rows(None, ctypes.byref(bc), None, 0, 1, None, ptr(offs), ctypes.byref(rec), None, ptr(st0), s)
    starts = torch.tensor([0, nrec], dtype=torch.int64, device=dev)

    def dedup():
        st = torch.zeros(68, dtype=torch.int64, device=dev)
        ok, oc = (torch.empty(nrec, dtype=torch.int64, device=dev) for _ in range(2))
        ng = torch.zeros(1, dtype=torch.int32, device=dev)
        sdp.sdp_part_dedup(ctypes.byref(rec), 1, ctypes.byref(bc), ptr(starts), 1, 1, ptr(ok), ptr(oc), ptr(ng),
                           ptr(st), s)
        return st.cpu().numpy()

    good = dedup()
    assert good[2] == 0 and good[3] == 0 and int(good[4:].sum()) == len(set(vals))
    # metas with row indices past the column (and one below it) on long and short keys
    bad_rows = torch.arange(0, nrec, 7, device=dev)
    meta[bad_rows] += 1 << 39
    meta[3] = meta[3] & ~((1 << 40) - 1)                 # row index -1
    bad = dedup()
    torch.cuda.synchronize()
    assert bad[2] != 0                                    # collision: the caller recounts exactly
    tab = e.value_counts_bytes_table(col)                 # the exact recount
    m = tab['groups']
    assert m == len(set(vals))
    assert int(tab['rows']) == n
    want = Counter(vals)
    assert sorted(want.values()) == sorted(int(c) for c in
                                           tab['counts'][:tab['capacity']].cpu().numpy() if c > 0)


def test_mixed_skewed_f32_and_timestamp_paths_chosen_once():
    """>= 8 numeric columns of 64 K - 2^26 rows -- five
    unskewed float32, three zipf-skewed high-cardinality float32 (heavy keys)
    and a timestamp column -- each take the distinct path describe() chose
    once, before pass 2 consumed the heavy-key samples, and match the oracle."""
    import oracle
    from spark_df_profiling import describe
    g = datagen.rng(41)
    n = 100_003
    cols = {}
    for k in range(5):
        cols['f32_u%d' % k] = pa.array(g.standard_normal(n).astype(np.float32), mask=g.random(n) < 0.03)
    for k in range(3):
        z = np.minimum(g.zipf(1.3 + 0.1 * k, n), 10 ** 7).astype(np.float32) + np.float32(0.5)
        cols['f32_z%d' % k] = pa.array(z)
    cols['ts'] = pa.array(g.integers(0, 10 ** 15, n), type=pa.timestamp('us'))
    t = pa.table(cols)
    assert_describe_equal(describe(t, plots=False), oracle.describe(t))
