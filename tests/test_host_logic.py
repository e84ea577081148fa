"""Host-side arithmetic of the engine vs the oracle (CPU only, no kernels)."""

import math
import random

import numpy as np
import pytest

import oracle.spark_describe as osd
from spark_df_profiling import engine as eng
from spark_df_profiling import _native as nat
from spark_df_profiling.utils import corr_from_gram, pretty_name


def test_pretty_name():
    assert [pretty_name(p) for p in (0.05, 0.25, 0.5, 0.75, 0.95)] == ['5%', '25%', '50%', '75%', '95%']
    assert pretty_name(0.125) == '12.5%'


@pytest.mark.parametrize('seed', range(20))
def test_hist_edges_match_oracle(seed):
    r = random.Random(seed)
    lo = r.uniform(-1e6, 1e6)
    hi = lo + abs(r.gauss(0, 10 ** r.randint(-3, 8)))
    bins = r.choice([2, 3, 7, 10, 33, 100])
    assert eng.hist_edges(lo, hi, bins) == osd.hist_edges(lo, hi, bins)


def test_hist_edges_bins_one():
    with pytest.raises(IndexError):
        eng.hist_edges(0.0, 1.0, 1)


@pytest.mark.parametrize('n', [1, 2, 3, 8, 9, 100, 9999, 10000, 10001, 123457])
def test_percentile_approx_rank(n):
    for p in (0.05, 0.25, 0.5, 0.75, 0.95, 1e-5, 0.99999):
        assert eng.spark_percentile_approx_rank(n, p) == osd.spark_percentile_approx_rank(n, p)


def _f64_key(x):
    b = np.array([0.0 if x == 0 else x], dtype=np.float64).view(np.uint64)[0]
    if x != x:
        b = np.uint64(0x7FF8000000000000)
    b = int(b)
    return (~b & ((1 << 64) - 1)) if b >> 63 else b | (1 << 63)


def test_key_roundtrip_and_order():
    vals = [-np.inf, -1e300, -2.5, -1.0, -5e-324, 0.0, 5e-324, 1.0, 3.5, 1e300, np.inf]
    keys = [_f64_key(v) for v in vals]
    assert keys == sorted(keys)
    assert _f64_key(float('nan')) > _f64_key(np.inf)
    assert _f64_key(-0.0) == _f64_key(0.0)
    for v, k in zip(vals, keys):
        assert eng.key_to_float(k) == v
    for i in (-2 ** 63, -1, 0, 1, 2 ** 63 - 1):
        assert eng.key_to_int((i & ((1 << 64) - 1)) ^ (1 << 63)) == i


def _p1_from(x, K, is_int):
    """What pass 1 accumulates, restated exactly (Fractions) for a data chunk."""
    from fractions import Fraction
    r = nat.SdpPass1Result()
    d = [Fraction(float(v)) - Fraction(K) for v in x]
    s1 = sum(d, Fraction(0))
    r.count = len(x)
    r.n_valid = len(x)
    r.shift = K
    r.s1_hi = float(s1)
    r.s1_lo = float(s1 - Fraction(r.s1_hi))
    r.s2 = float(sum((t * t for t in d), Fraction(0)))
    s3 = sum((t * t * t for t in d), Fraction(0))
    r.s3_hi = float(s3)
    r.s3_lo = float(s3 - Fraction(r.s3_hi))
    r.s4 = float(sum((t ** 4 for t in d), Fraction(0)))
    if is_int:
        r.isum = int(np.sum(np.asarray(x, dtype=np.int64)))
        r.imin, r.imax = int(min(x)), int(max(x))
    else:
        r.dmin, r.dmax = float(min(x)), float(max(x))
    return r


@pytest.mark.parametrize('kind', ['norm', 'shifted', 'lognormal', 'int'])
def test_moments_from_power_sums_match_oracle(kind):
    g = np.random.default_rng(3)
    if kind == 'norm':
        x = g.standard_normal(4000)
    elif kind == 'shifted':
        x = 1e9 + g.standard_normal(4000)
    elif kind == 'lognormal':
        x = g.lognormal(3, 2, 4000)
    else:
        x = g.integers(-10 ** 6, 10 ** 6, 4000)
    is_int = kind == 'int'
    K = float(np.median(x))
    parts = [_p1_from(c, K, is_int) for c in np.array_split(x, 3)]
    p1 = eng.merge_pass1_results(parts)
    got = eng.moments(p1, is_int)
    want = osd.numeric_stats(np.asarray(x), np.ones(len(x), bool), is_int, len(x), 10, 2)
    for k in ('mean', 'variance', 'std', 'skewness', 'kurtosis', 'sum', 'min', 'max'):
        assert math.isclose(got[k], want[k], rel_tol=1e-12, abs_tol=1e-12), (k, got[k], want[k])


def test_int_sum_wraps():
    parts = [_p1_from([2 ** 62, 2 ** 62], 0.0, True), _p1_from([2 ** 62, 5], 0.0, True)]
    p1 = eng.merge_pass1_results(parts)
    assert p1['isum'] == (3 * 2 ** 62 + 5) - 2 ** 64


def test_corr_from_gram():
    g = np.random.default_rng(1)
    X = g.standard_normal((500, 4))
    X[:, 1] += X[:, 0]
    K = X.mean(0) + 0.3
    Xc = X - K
    rho = corr_from_gram(Xc.T @ Xc, Xc.sum(0), len(X))
    assert np.allclose(rho, np.corrcoef(X.T), rtol=1e-12, atol=1e-12)
    assert np.isnan(corr_from_gram(np.zeros((2, 2)), np.zeros(2), 0)).all()


def test_spark_to_arrow_duck_types():
    """describe.spark_to_arrow on Spark-like objects of each collect style
    (no GPU: the Arrow table is returned before any upload)."""
    import pyarrow as pa
    from spark_df_profiling.describe import spark_to_arrow
    t = pa.table({'a': pa.array([1, 2, None]), 's': pa.array(['x', None, 'z'])})

    class S4:
        def toArrow(self):
            return t

    class S3:
        def _collect_as_arrow(self):
            return t.to_batches(max_chunksize=2)

    class S2:
        def toPandas(self):
            return t.to_pandas()

    assert spark_to_arrow(S4()).equals(t)
    assert spark_to_arrow(S3()).equals(t)
    got = spark_to_arrow(S2())
    assert got.column('s').to_pylist() == ['x', None, 'z']
    assert got.column('a').to_pylist()[:2] == [1.0, 2.0]


def test_sample_nondecreasing_flags():
    import torch
    from spark_df_profiling.engine import Engine
    E = -1                                            # UINT64_MAX: a null / NaN sample row
    big = (1 << 63) + 5                               # keys above 2^63 (positive floats' keys)
    rows = [[1, 2, 2, E, 3, 9],                       # non-decreasing with a null
            [1, 3, 2, 4, 5, 6],                       # one decrease
            [E, E, 7, E, E, E],                       # one valid key: not a candidate
            [5, big - (1 << 64), E, big + 1 - (1 << 64), E, E],   # across the sign bit, unsigned order
            [big - (1 << 64), 5, 6, 7, 8, 9]]         # big key first: decreasing in unsigned order
    t = torch.tensor(rows, dtype=torch.int64)
    assert Engine._sample_nondecreasing(t).tolist() == [1, 0, 0, 1, 0]


def test_merge_sorted_distinct_rank_order():
    import numpy as np
    from spark_df_profiling.engine import merge_sorted_distinct
    E = np.uint64(2 ** 64 - 1)
    p = lambda d, v, f, l: np.array([d, v, f, l], dtype=np.uint64)
    assert merge_sorted_distinct([p(5, 0, 10, 20)]) == 5
    # rank boundary with an equal key: one value, counted once
    assert merge_sorted_distinct([p(5, 0, 10, 20), p(3, 0, 20, 30)]) == 7
    assert merge_sorted_distinct([p(5, 0, 10, 20), p(3, 0, 21, 30)]) == 8
    # an empty rank in between is skipped; a decrease across ranks is not sorted
    assert merge_sorted_distinct([p(5, 0, 10, 20), p(0, 0, E, E), p(1, 0, 20, 20)]) == 5
    assert merge_sorted_distinct([p(5, 0, 10, 20), p(3, 0, 19, 30)]) is None
    assert merge_sorted_distinct([p(5, 1, 10, 20)]) is None


def test_select_sizing_mirrors_the_library():
    """quantiles_batch sizes select workspaces and radix rounds on the host
    (Engine._select_ws / _select_rounds); they must equal the C ABI's
    sdp_select_kth_workspace_bytes / sdp_select_rounds (no GPU needed)."""
    import random
    from spark_df_profiling.engine import Engine
    from spark_df_profiling._native import sdp
    for n in [0, 1, 2, 31, 32, 33, 1000, 12345678, 10 ** 9]:
        assert Engine._select_ws(n) == sdp.sdp_select_kth_workspace_bytes(n), n
    rnd = random.Random(3)
    for _ in range(2000):
        lo = rnd.getrandbits(64)
        hi = rnd.getrandbits(rnd.randint(0, 64))
        assert Engine._select_rounds(lo, hi) == sdp.sdp_select_rounds(lo, hi)



def test_fusable_groups_wide_tables_only():
    """group_batch fuses the scans, level-1 scatters, level-2 and dedup stages
    of >= FUSE_MIN_COLS small fixed-key, distinct-only columns of one geometry
    and dtype (Engine._fusable, decided before the scans); byte keys, counted
    groups, single-level, empty and large columns stay single."""
    from spark_df_profiling.engine import Engine
    e = Engine(device='cpu')

    class Col:
        def __init__(self, n, dtype=9):
            self.length, self.dtype = n, dtype

    def ctx(n=10 ** 7, b1=7, b2=7, isb=False, wc=False, large=False, dtype=9):
        return {'isb': isb, 'with_counts': wc, 'large': large, 'b1': b1, 'b2': b2, 'col': Col(n, dtype)}

    ctxs = [ctx() for _ in range(10)] + [ctx(isb=True), ctx(wc=True), ctx(b2=0), ctx(b1=8), ctx(n=0), ctx(dtype=8)]
    fuse, single = e._fusable(ctxs)
    assert fuse == [list(range(10))]
    assert single == [10, 11, 12, 13, 14, 15]
    fuse, single = e._fusable([ctx(n=10 ** 8) for _ in range(9)])          # 1e8 rows each: not fused
    assert fuse == [] and single == list(range(9))
    fuse, single = e._fusable([ctx() for _ in range(5)])                   # too few columns
    assert fuse == [] and single == list(range(5))
    e.FUSE_BYTES = 16 * 3 * 10 ** 7                                        # three columns per group
    fuse, single = e._fusable([ctx() for _ in range(8)])
    assert fuse == [[0, 1, 2], [3, 4, 5], [6, 7]] and single == []


def test_spark_batches_and_stream_inputs():
    """describe.spark_batches / _batch_stream (no GPU: nothing is uploaded):
    Spark-like objects of each transfer style and plain batch streams give
    (schema, batches, rows or None); an iterator is not consumed up front."""
    import pyarrow as pa
    from spark_df_profiling.describe import _batch_stream, spark_batches
    t = pa.table({'a': pa.array([1, 2, None, 4, 5]), 's': pa.array(['x', None, 'z', 'w', 'v'])})

    class S4:
        def toArrow(self):
            return t

    class S3:
        def _collect_as_arrow(self):
            return t.to_batches(max_chunksize=2)

    class S3It:
        pulled = 0

        def _collect_as_arrow(self):
            for b in t.to_batches(max_chunksize=2):
                S3It.pulled += 1
                yield b

    sch, bs, rows = spark_batches(S4())
    assert sch == t.schema and rows == 5 and pa.Table.from_batches(list(bs)).equals(t)
    sch, bs, rows = spark_batches(S3())
    assert rows == 5 and pa.Table.from_batches(list(bs)).equals(t)
    sch, bs, rows = spark_batches(S3It())
    assert rows is None and sch == t.schema and S3It.pulled == 1       # only the first batch peeked
    assert pa.Table.from_batches(list(bs)).equals(t) and S3It.pulled == 3
    assert _batch_stream([1, 2]) is None and _batch_stream(iter([1])) is None
    rd = pa.RecordBatchReader.from_batches(t.schema, t.to_batches(max_chunksize=3))
    assert _batch_stream(rd)[2] is None


def test_apply_spark_dtypes_cpu():
    import pyarrow as pa
    import pytest
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.describe import apply_spark_dtypes
    t = pa.table({'a': pa.array([1, 2, 3], pa.int64()), 's': pa.array(['x', 'y', 'z'])})
    dt = DeviceTable.from_arrow(t, device='cpu', streamed=False)
    apply_spark_dtypes(dt, {'a': 'bigint', 's': 'string'})
    assert [c.spark_type for c in dt.columns] == ['bigint', 'string']
    with pytest.raises(TypeError):
        apply_spark_dtypes(dt, {'s': 'double'})
