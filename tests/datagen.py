"""Seeded Arrow tables for the parity tests (numpy PCG64, fixed seeds)."""

import datetime
import decimal

import numpy as np
import pyarrow as pa


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def legacy_table():
    """tests.py.old.py:23-37 data as Spark would type it:
    x bigint with a null, y double with a null, somedate timestamp."""
    return pa.table({
        'id': pa.array([chr(97 + c) for c in range(1, 10)]),
        'x': pa.array([50, 50, -10, 0, 0, 5, 15, -3, None], pa.int64()),
        'y': pa.array([0.000001, 654.152, None, 15.984512, 3122, -3.1415926535, 111, 15.9, 13.5], pa.float64()),
        'cat': pa.array(['a', 'long text value', u'Élysée', '', None, 'some <b> B.s </div> </div> HTML stuff',
                         'c', 'c', 'c']),
        's1': pa.array(np.ones(9)),
        's2': pa.array([u'some constant text $ % value {obj} ' for _ in range(1, 10)]),
        'somedate': pa.array([datetime.datetime(2011, 7, 4), datetime.datetime(2022, 1, 1, 13, 57),
                              datetime.datetime(1990, 12, 9), None, datetime.datetime(1990, 12, 9),
                              datetime.datetime(1950, 12, 9), datetime.datetime(1898, 1, 2),
                              datetime.datetime(1950, 12, 9), datetime.datetime(1950, 12, 9)],
                             pa.timestamp('us')),
    })


def legacy_table_pandas_typed():
    """The same data typed as pandas -> Spark would: x double with NaN."""
    t = legacy_table()
    x = pa.array([50.0, 50.0, -10.0, 0.0, 0.0, 5.0, 15.0, -3.0, float('nan')], pa.float64())
    return t.set_column(t.schema.get_field_index('x'), 'x', x)


def _mask(g, n, p):
    return g.random(n) < p


def numeric_table(n, seed=20261015, null_p=0.05):
    g = rng(seed)
    cols = {}
    cols['f64_norm'] = g.standard_normal(n)
    cols['f64_shift'] = 1e9 + g.standard_normal(n)
    cols['f64_logn'] = g.lognormal(3, 2, n)
    f = g.standard_normal(n)
    f[_mask(g, n, 0.01)] = np.nan
    f[_mask(g, n, 0.02)] = 0.0
    f[_mask(g, n, 0.005)] = -0.0
    cols['f64_nan_zero'] = f
    cols['f32_unif'] = g.random(n).astype(np.float32)
    cols['i64_small'] = g.integers(0, 1000, n)
    cols['i64_wide'] = g.integers(-2 ** 31, 2 ** 31, n)
    cols['i64_zipf'] = np.minimum(g.zipf(1.3, n), 10 ** 6).astype(np.int64)
    cols['i32_seq'] = np.arange(n, dtype=np.int32)
    cols['i16'] = g.integers(-300, 300, n).astype(np.int16)
    cols['i8'] = g.integers(-128, 128, n).astype(np.int8)
    cols['u8'] = g.integers(0, 256, n).astype(np.uint8)
    cols['u32'] = g.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
    out = {}
    for k, v in cols.items():
        m = _mask(g, n, null_p) if k not in ('i32_seq',) else None
        out[k] = pa.array(v, mask=m)
    # heavy ties at the quartiles: 40% one value
    h = g.standard_normal(n)
    h[_mask(g, n, 0.4)] = 1.5
    out['f64_heavy'] = pa.array(h)
    return pa.table(out)


def small_edge_table():
    """Edge cases the reference's semantics define (App. C)."""
    return pa.table({
        'const_int': pa.array([7] * 6, pa.int64()),
        'const_float_nan': pa.array([np.nan, 2.0, np.nan, 2.0, 2.0, np.nan], pa.float64()),
        'all_null': pa.array([None] * 6, pa.int32()),
        'all_nan': pa.array([np.nan] * 6, pa.float64()),
        'two_vals': pa.array([1, 2, 1, 2, 1, 2], pa.int16()),
        'one_valid': pa.array([None, None, 3.5, None, np.nan, None], pa.float64()),
        'neg_zero': pa.array([0.0, -0.0, 1.0, -1.0, 0.0, 2.0], pa.float64()),
        'int_extremes': pa.array([2 ** 63 - 1, -2 ** 63, 0, 1, -1, 5], pa.int64()),
        'bools': pa.array([True, False, None, True, True, False], pa.bool_()),
        'nulltype': pa.nulls(6),
    })


def wide_range_table(n=4099, seed=53):
    """Columns whose histogram range depends on the type the min / max have at
    describe.py:211 / :226: stats_df.ix[0] (:209) upcasts
    the agg row to float64, so the range and the accumulated edges are float64
    arithmetic on float64(min) / float64(max) -- not int64 (|min|, |max| >
    2^53 here, where float(int(max) - int(min)) rounds differently) and not
    float32 (max - min rounds to another float32).  The int64 sum wraps."""
    g = rng(seed)
    big = g.integers(-(2 ** 60), 2 ** 61, n, dtype=np.int64)
    big[0], big[1] = 2 ** 61 + 200, -(2 ** 60) - 200            # max / min
    big[6:40] = 2 ** 61 + 100 - np.arange(34)                    # many values near the top edges
    f32 = (g.standard_normal(n) * 1e3).astype(np.float32)
    f32[0], f32[1] = np.float32(1.0e8), np.float32(-3.3333333)
    # values right at the float64 edges of the float32 column
    lo, hi = float(np.float32(-3.3333333)), float(np.float32(1.0e8))
    w = (hi - lo) / 10.0
    e, edges = lo, []
    for _ in range(10):
        edges.append(e)
        e += w
    f32[2:12] = np.array(edges, dtype=np.float32)
    wrap = np.full(n, 2 ** 62, dtype=np.int64)                   # sum wraps past 2^63 several times
    wrap[::3] = -(2 ** 61)
    m = _mask(g, n, 0.03)
    m[:12] = False
    return pa.table({'i64_big': pa.array(big, mask=m), 'f32_range': pa.array(f32, mask=m),
                     'i64_wrap': pa.array(wrap, mask=m)})


def categorical_table(n, seed=7, card=(100, 5000)):
    g = rng(seed)
    words = np.array(['w%05d_%s' % (i, 'x' * (i % 13)) for i in range(max(card))], dtype=object)
    out = {}
    z = np.minimum(g.zipf(1.2, n), card[0]) - 1
    out['cat_zipf'] = pa.array(words[z], mask=_mask(g, n, 0.05))
    u = g.integers(0, card[1], n)
    out['cat_unif'] = pa.array(words[u])
    out['cat_big'] = pa.array(['u%d' % i for i in g.permutation(n)])          # UNIQUE
    out['cat_two'] = pa.array(np.where(g.random(n) < 0.7, 'Found', 'Fell').astype(object), mask=_mask(g, n, 0.01))
    out['cat_empty'] = pa.array(np.where(g.random(n) < 0.5, '', 'Élysée').astype(object))
    out['bool'] = pa.array(g.random(n) < 0.3, mask=_mask(g, n, 0.1))
    out['large'] = pa.array(words[z].tolist(), type=pa.large_string())
    out['bin'] = pa.array([w.encode() for w in words[u]], type=pa.binary())
    out['dec'] = pa.array([decimal.Decimal(int(x)).scaleb(-2) for x in g.integers(-500, 500, n)],
                          type=pa.decimal128(10, 2))
    out['num'] = pa.array(g.integers(0, 50, n))     # describe.py:108 needs one NUM column
    return pa.table(out)


def date_table(n, seed=11):
    g = rng(seed)
    days = g.integers(-100000, 50000, n).astype(np.int32)
    ts = g.integers(-2 * 10 ** 15, 2 * 10 ** 15, n)
    return pa.table({
        'd': pa.array(days, type=pa.date32(), mask=_mask(g, n, 0.05)),
        'ts': pa.array(ts, type=pa.timestamp('us'), mask=_mask(g, n, 0.05)),
        'num': pa.array(g.standard_normal(n)),
    })


def corr_table(n, seed=5):
    g = rng(seed)
    a = g.standard_normal(n)
    b = a + 0.1 * g.standard_normal(n)             # rho ~ 0.995 -> CORR
    c = -a + g.standard_normal(n)
    d = g.random(n).astype(np.float32)
    e = (100 * a).astype(np.int64)
    return pa.table({'a': pa.array(a, mask=_mask(g, n, 0.03)), 'b': pa.array(b), 'c': pa.array(c),
                     'd': pa.array(d, mask=_mask(g, n, 0.03)), 'e': pa.array(e)})


def demo_like_table(n, seed=20261015):
    """Config-1 column mix: Demo.ipynb-style meteorites."""
    g = rng(seed)
    labels = np.array(['L%03d' % i for i in range(466)], dtype=object)
    reclat = g.uniform(-90, 90, n)
    reclat[_mask(g, n, 0.14)] = 0.0
    rmask = _mask(g, n, 0.19)
    days = (g.integers(1688, 2102, n) - 1970) * 365
    return pa.table({
        'name': pa.array(['name%d' % i for i in range(n)]),
        'id': pa.array(np.arange(n, dtype=np.int64)),
        'nametype': pa.array(np.where(g.random(n) < 0.998, 'Valid', 'Relict').astype(object)),
        'recclass': pa.array(labels[np.minimum(g.zipf(1.3, n), 466) - 1]),
        'mass_g': pa.array(g.lognormal(3, 2, n), mask=_mask(g, n, 0.003)),
        'fall': pa.array(np.where(g.random(n) < 0.976, 'Found', 'Fell').astype(object)),
        'reclat': pa.array(reclat, mask=rmask),
        'reclat_city': pa.array(reclat + g.standard_normal(n), mask=rmask),
        'source': pa.array(['NASA'] * n),
        'year': pa.array(days.astype(np.int32), type=pa.date32(), mask=_mask(g, n, 0.007)),
    })


# ----------------------------------------------------------------------------
# BASELINE.json configurations, numpy PCG64 from fixed seeds.
# C1 is demo_like_table above; C3 is generated in HBM by bench.make_c3_shard.
# ----------------------------------------------------------------------------

C_SEED = 20261015


def c2_table(n, seed=C_SEED):
    """C2: n x 8 fp64, no nulls -- N(0,1), N(1e9,1) (cancellation stress),
    lognormal(0,1), U(-1e6,1e6), exp(1), Student-t(3), 1 % exact zeros + N(0,1),
    bimodal."""
    g = rng(seed)
    z = g.standard_normal(n)
    z[g.random(n) < 0.01] = 0.0
    bi = np.where(g.random(n) < 0.3, g.normal(-5.0, 1.0, n), g.normal(4.0, 0.5, n))
    cols = {
        'norm': g.standard_normal(n),
        'shifted_1e9': 1e9 + g.standard_normal(n),
        'lognormal': g.lognormal(0.0, 1.0, n),
        'uniform_1e6': g.uniform(-1e6, 1e6, n),
        'exp': g.exponential(1.0, n),
        'student_t3': g.standard_t(3, n),
        'zeros_1pct': z,
        'bimodal': bi,
    }
    return pa.table({k: pa.array(v) for k, v in cols.items()})


def bounded_zipf(g, n, s, card):
    """Continuous power-law inverse CDF on [1, card+1) -> labels 0..card-1
    (the same law bench.py draws its zipf columns from)."""
    u = g.random(n)
    a = 1.0 - s
    x = np.power(1.0 - u * (1.0 - (card + 1.0) ** a), 1.0 / a)
    return np.clip(np.floor(x).astype(np.int64) - 1, 0, card - 1)


def mix64_np(x):
    x = np.asarray(x, dtype=np.uint64).copy()
    with np.errstate(over='ignore'):
        x ^= x >> np.uint64(30)
        x *= np.uint64(0xBF58476D1CE4E5B9)
        x ^= x >> np.uint64(27)
        x *= np.uint64(0x94D049BB133111EB)
        x ^= x >> np.uint64(31)
    return x


def hex16_strings(keys):
    """utf8 array of the 16 lower-case hex digits of each u64 key."""
    keys = np.asarray(keys, dtype=np.uint64)
    n = keys.size
    shifts = np.arange(60, -4, -4, dtype=np.uint64)
    nib = ((keys[:, None] >> shifts[None, :]) & np.uint64(15)).astype(np.uint8)
    data = np.frombuffer(b'0123456789abcdef', dtype=np.uint8)[nib].reshape(-1)
    offsets = (np.arange(n + 1, dtype=np.int32) * 16)
    return pa.StringArray.from_buffers(n, pa.py_buffer(offsets.tobytes()), pa.py_buffer(data.tobytes()))


def c4_table(n, seed=C_SEED + 4, labels=5 * 10 ** 8):
    """C4: int64 U[0, 2^32) (near-unique) and utf8 16-byte hex ids drawn
    zipf(1.05) over `labels` labels (exact distinct + top-50), plus the NUM
    column the reference needs for table stats (describe.py:108)."""
    g = rng(seed)
    ints = g.integers(0, 2 ** 32, n, dtype=np.int64)
    lab = bounded_zipf(g, n, 1.05, labels)
    return pa.table({'u32_range_i64': pa.array(ints), 'hex_id': hex16_strings(mix64_np(lab))})


def c5_table(n, ncols=512, seed=C_SEED + 5, factors=4):
    """C5: n x ncols fp32, no nulls: x_j = F a_j + e_j, F ~ N(0,1) (n x 4),
    loadings a_j ~ U(-1.5, 1.5)^4, so the Pearson matrix spans (-1, 1)."""
    g = rng(seed)
    F = g.standard_normal((n, factors))
    L = g.uniform(-1.5, 1.5, (factors, ncols))
    cols = {}
    for j in range(ncols):
        cols['c%03d' % j] = pa.array((F @ L[:, j] + g.standard_normal(n)).astype(np.float32))
    return pa.table(cols)


def sorted_table(n, seed=41):
    """Columns sorted in row order (ids, timestamps, pre-sorted data) and
    near-misses, for the sorted-column countDistinct path (sdp_sorted_distinct):
    strictly increasing ids with nulls, non-decreasing values with duplicates,
    sorted doubles with -0.0/+0.0 and NaN at the end, one swapped pair deep
    inside, a null run longer than the kernel's walk, a descending column."""
    g = rng(seed)
    ids = np.arange(n, dtype=np.int64) * 3 + 7
    dup = np.sort(g.integers(0, max(2, n // 10), n)).astype(np.int64)
    f = np.sort(g.standard_normal(n))
    z = int(np.searchsorted(f, 0.0))                      # -0.0 then +0.0 where the values cross zero
    f[z - 25:z] = -0.0
    f[z:z + 25] = 0.0
    h = n // 2
    f[h:h + 10] = f[h + 10]                               # a small tie run
    f[-(n // 100):] = np.nan                              # NaN sorts last (countDistinct: one value)
    almost = np.arange(n, dtype=np.int64)
    almost[n // 2], almost[n // 2 + 1] = almost[n // 2 + 1], almost[n // 2]
    runs = np.arange(n, dtype=np.float64)
    rmask = np.zeros(n, dtype=bool)
    rmask[n // 4: n // 4 + 1000] = True                   # a null run longer than the walk (256)
    return pa.table({
        'ids': pa.array(ids, mask=_mask(g, n, 0.05)),
        'dup': pa.array(dup, mask=_mask(g, n, 0.03)),
        'fsort': pa.array(f, mask=_mask(g, n, 0.02)),
        'f32sort': pa.array(np.sort(g.random(n)).astype(np.float32)),
        'almost': pa.array(almost),
        'nullrun': pa.array(runs, mask=rmask),
        'desc': pa.array(np.arange(n, dtype=np.int64)[::-1].copy()),
        'num': pa.array(g.standard_normal(n)),
    })
