"""numpy/pyarrow restatement of the reference statistics engine -- TEST INFRASTRUCTURE ONLY.

Every function below names the reference lines it follows.  Spark SQL arithmetic
that the reference delegates to (not present under /root/reference) is restated
from SURVEY.md Appendix A ([upstream], Spark 2.x):

* A.1 Average: double sum / count           * A.2 Sum: int64 wraps, else double
* A.3 CentralMomentAgg: var_samp, stddev_samp, skewness, kurtosis (population)
* A.4 Percentile (exact, int columns)         * A.5 ApproximatePercentile -> the
  element at 1-based rank ceil(p*N) (defined contract)
* A.6 histogram edges accumulated on the host * A.7 Corr (Pearson, listwise)
  -- from float64 min / max for every column type: describe.py:209
  `stats_df.ix[0]` upcasts the mixed int64 / float32 / float64 agg row to one
  float64 Series before :211 (range) and :226 (edges), which overrides A.6's
  int64 / float32 subtraction (tests/test_oracle_golden.py pins it on
  datagen.wide_range_table: |min|, |max| > 2^53 and a float32 range that
  rounds differently)
* A.8 NaN/null: na.drop drops null and NaN; countDistinct counts NaN once;
  NaN orders above every number; -0.0 groups with 0.0 (3.x, recorded choice).

The oracle aims at the *exact* value of each statistic (math.fsum, exact sorts),
so that the HIP path is judged against truth, not against another rounding order.
"""

from __future__ import annotations

import datetime as _dt
import math
from collections import OrderedDict

import numpy as np
import pandas as pd
import pyarrow as pa

# ----------------------------------------------------------------------------
# Spark type strings (describe.py:137 `df.select(column).dtypes[0][1]`)
# ----------------------------------------------------------------------------

_INT_TYPES = ('tinyint', 'smallint', 'int', 'bigint')      # describe.py:158
_FLOAT_TYPES = ('float', 'double', 'decimal')              # describe.py:160
_DATE_TYPES = ('date', 'timestamp')                        # describe.py:162


def spark_type_of(t: pa.DataType) -> str:
    """Arrow type -> the Spark SQL simpleString the reference dispatches on."""
    if pa.types.is_dictionary(t):
        return spark_type_of(t.value_type)
    if pa.types.is_int8(t):
        return 'tinyint'
    if pa.types.is_int16(t) or pa.types.is_uint8(t):
        return 'smallint'
    if pa.types.is_int32(t) or pa.types.is_uint16(t):
        return 'int'
    if pa.types.is_int64(t) or pa.types.is_uint32(t):
        return 'bigint'
    if pa.types.is_uint64(t):
        return 'decimal(20,0)'
    if pa.types.is_float16(t) or pa.types.is_float32(t):
        return 'float'
    if pa.types.is_float64(t):
        return 'double'
    if pa.types.is_decimal(t):
        return 'decimal(%d,%d)' % (t.precision, t.scale)
    if pa.types.is_boolean(t):
        return 'boolean'
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        return 'string'
    if pa.types.is_binary(t) or pa.types.is_large_binary(t) or pa.types.is_fixed_size_binary(t):
        return 'binary'
    if pa.types.is_date(t):
        return 'date'
    if pa.types.is_timestamp(t):
        return 'timestamp'
    if pa.types.is_null(t):
        return 'null'
    if pa.types.is_list(t) or pa.types.is_large_list(t) or pa.types.is_fixed_size_list(t):
        return 'array<%s>' % spark_type_of(t.value_type)
    if pa.types.is_struct(t):
        return 'struct<%s>' % ','.join('%s:%s' % (f.name, spark_type_of(f.type)) for f in t)
    if pa.types.is_map(t):
        return 'map<%s,%s>' % (spark_type_of(t.key_type), spark_type_of(t.item_type))
    raise NotImplementedError('Arrow type %s has no Spark SQL counterpart' % t)


# ----------------------------------------------------------------------------
# helpers
# ----------------------------------------------------------------------------

def pretty_name(x):
    """utils.py:7-12"""
    x *= 100
    if x == int(x):
        return '%.0f%%' % x
    return '%.1f%%' % x


def fmt_bytesize(num, suffix='B'):
    """formatters.py:29-34"""
    for unit in ['', 'Ki', 'Mi', 'Gi', 'Ti', 'Pi', 'Ei', 'Zi']:
        if abs(num) < 1024.0:
            return "%3.1f %s%s" % (num, unit, suffix)
        num /= 1024.0
    return "%.1f %s%s" % (num, 'Yi', suffix)


def _fsum(a):
    a = np.asarray(a, dtype=np.float64)
    if a.size == 0:
        return 0.0
    if not np.all(np.isfinite(a)):
        return float(np.sum(a))
    return math.fsum(a.tolist())


_CHUNK = 1 << 16


def _sum(a, fast=False):
    """Exact sum (math.fsum) or, in the vectorised mode, numpy's pairwise sum
    of 64 K-element chunks added exactly: error <= ~16 eps * sum|a|, far inside
    the 1e-9 relative parity bound for every statistic built from it."""
    if not fast:
        return _fsum(a)
    a = np.asarray(a, dtype=np.float64)
    if a.size == 0:
        return 0.0
    if a.size <= _CHUNK:
        return float(np.sum(a))
    m = a.size // _CHUNK * _CHUNK
    parts = np.sum(a[:m].reshape(-1, _CHUNK), axis=1).tolist()
    parts.append(float(np.sum(a[m:])))
    if not all(math.isfinite(x) for x in parts):
        return float(np.sum(parts))
    return math.fsum(parts)


def _spark_gt(x, t):
    """Spark `x > t` with NaN ordered above every number (A.8)."""
    x = np.asarray(x, dtype=np.float64)
    if math.isnan(t):
        return np.zeros(x.shape, bool)
    return np.isnan(x) | (x > t)


def _spark_lt(x, t):
    x = np.asarray(x, dtype=np.float64)
    if math.isnan(t):
        return ~np.isnan(x)
    return (~np.isnan(x)) & (x < t)


def _spark_ge(x, t):
    return ~_spark_lt(x, t)


def _column(table, name):
    col = table.column(name)
    if isinstance(col, pa.ChunkedArray):
        col = col.combine_chunks() if col.num_chunks != 1 else col.chunk(0)
    if pa.types.is_dictionary(col.type):
        col = col.dictionary_decode()
    return col


def _valid_mask(arr):
    if arr.null_count == 0:
        return np.ones(len(arr), bool)
    return np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), bool)


def _numeric_values(arr, spark_t):
    """Values with nulls filled; ints as int64, floats as float64 (exact upcast)."""
    if spark_t in _INT_TYPES:
        return np.asarray(arr.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.int64)
    return np.asarray(arr.fill_null(0).to_numpy(zero_copy_only=False)).astype(np.float64)


def _canon_float_keys(x):
    """countDistinct grouping keys: NaN once, -0.0 == 0.0 (A.8)."""
    x = np.where(x == 0.0, 0.0, x)
    bits = x.view(np.uint64).copy()
    bits[np.isnan(x)] = np.uint64(0x7FF8000000000000)
    return bits


# ----------------------------------------------------------------------------
# numeric statistics (describe.py:192-229)
# ----------------------------------------------------------------------------

def hist_edges(minim, maxim, bins):
    """describe.py:40-45 -- edges by *accumulated* addition, last one popped."""
    num_range = maxim - minim
    bin_width = num_range / float(bins)
    left_edges = [minim]
    for _bin in range(bins):
        left_edges = left_edges + [left_edges[-1] + bin_width]
    left_edges.pop()
    if len(left_edges) < 2:
        # describe.py:46 indexes left_edges[1]: bins=1 raises IndexError
        raise IndexError('list index out of range')
    return left_edges, bin_width


def hist_counts(xs, edges):
    """The CASE-WHEN chain of describe.py:46 + create_all_conditions :20-35,
    first matching branch wins; rows matching none (x < e0) get bin null and are
    dropped by the reindex at :53-57."""
    xs = np.asarray(xs, dtype=np.float64)
    b = len(edges)
    out = np.zeros(b, np.int64)
    unassigned = np.ones(xs.shape, bool)
    for i in range(b):
        if i < b - 1:
            cond = _spark_ge(xs, float(edges[i])) & _spark_lt(xs, float(edges[i + 1]))
        else:
            cond = _spark_ge(xs, float(edges[i]))
        hit = cond & unassigned
        out[i] = int(hit.sum())
        unassigned &= ~hit
    return out


def spark_percentile_exact(sorted_x, p, n=None):
    """Spark `percentile` (A.4), used for int columns (describe.py:203-204).
    `sorted_x` is the sorted column or a {rank: value} map of the two ranks
    this p needs (then n is the column length)."""
    n = len(sorted_x) if n is None else n
    position = (n - 1) * p
    lower = math.floor(position)
    higher = math.ceil(position)
    lower_key = sorted_x[lower]
    if higher == lower:
        return float(lower_key)
    higher_key = sorted_x[higher]
    if higher_key == lower_key:
        return float(lower_key)
    return (higher - position) * float(lower_key) + (position - lower) * float(higher_key)


def spark_percentile_approx_rank(n, p, relative_error=1e-4):
    """1-based rank of the element returned for float columns (A.5)."""
    if p <= relative_error:
        return 1
    if p >= 1 - relative_error:
        return n
    return min(max(int(math.ceil(p * n)), 1), n)


def _order_stats(x, ranks, fast):
    """{rank: value} of 0-based order statistics of x (stable sort, or an
    introselect partition at the needed ranks in the vectorised mode)."""
    ranks = sorted(set(int(r) for r in ranks))
    if not fast:
        sx = np.sort(x, kind='stable')
        return {r: sx[r] for r in ranks}
    px = np.partition(x, ranks)
    return {r: px[r] for r in ranks}


def numeric_stats(values, valid, is_int, nrows, bins, k, fast=False):
    """All of describe_numeric_1d (describe.py:192-229) except the PNGs.

    Returns an OrderedDict in the reference's key order plus '_hist' (counts,
    edges, width) for the bit-exact histogram checks.
    """
    v = values[valid]
    if is_int:
        xs_int = v
        xs = v.astype(np.float64)
    else:
        xs = v[~np.isnan(v)]
    n = len(xs)
    st = OrderedDict()
    # mean/min/max/variance/kurtosis/std/skewness/sum (:193-201)
    if is_int:
        mean = _sum(xs, fast) / n
        mn, mx = float(xs_int.min()), float(xs_int.max())
        total = float(np.sum(xs_int, dtype=np.int64))          # LongType wraps (A.2)
    else:
        mean = _sum(xs, fast) / n
        mn, mx = float(xs.min()), float(xs.max())
        total = _sum(xs, fast)
    d = xs - mean
    d2 = d * d
    c, s2, s3, s4 = _sum(d, fast), _sum(d2, fast), _sum(d2 * d, fast), _sum(d2 * d2, fast)
    del d2
    m2 = s2 - c * c / n
    m3 = s3 - 3.0 * c * s2 / n + 2.0 * c ** 3 / n ** 2
    m4 = s4 - 4.0 * c * s3 / n + 6.0 * c * c * s2 / n ** 2 - 3.0 * c ** 4 / n ** 3
    variance = float('nan') if n == 1 else m2 / (n - 1.0)
    std = float('nan') if n == 1 else math.sqrt(max(variance, 0.0))
    skew = float('nan') if m2 == 0 else math.sqrt(n) * m3 / math.sqrt(m2 * m2 * m2)
    kurt = float('nan') if m2 == 0 else n * m4 / (m2 * m2) - 3.0
    st['mean'] = mean
    st['min'] = mn
    st['max'] = mx
    st['variance'] = variance
    st['kurtosis'] = kurt
    st['std'] = std
    st['skewness'] = skew
    st['sum'] = total
    # percentiles (:203-208)
    probs = [0.05, 0.25, 0.5, 0.75, 0.95]
    if is_int:
        need = [r for p in probs for r in (math.floor((n - 1) * p), math.ceil((n - 1) * p))]
    else:
        need = [spark_percentile_approx_rank(n, p) - 1 for p in probs]
    sx = _order_stats(xs_int if is_int else xs, need, fast)
    qs = {}
    for p in probs:
        if is_int:
            q = spark_percentile_exact(sx, p, n)
        else:
            q = float(sx[spark_percentile_approx_rank(n, p) - 1])
        qs[p] = q
        st[pretty_name(p)] = q
    # derived (:211-214), numpy float64 semantics (division by zero -> inf/nan)
    with np.errstate(all='ignore'):
        st['range'] = np.float64(mx) - np.float64(mn)
        q3, q1 = qs[0.75], qs[0.25]
        st['iqr'] = np.float64(q3) - np.float64(q1)
        st['cv'] = np.float64(std) / float(mean)
        # mad (:215-218): *mean* absolute deviation around the Spark mean
        st['mad'] = np.float64(_sum(np.abs(xs - mean), fast)) / float(n)
    st['type'] = 'NUM'
    # zeros (:220-221) over the full column (null excluded, NaN != 0, -0.0 == 0)
    vd = values[valid].astype(np.float64)
    st['n_zeros'] = int(np.sum(vd == 0.0))
    st['p_zeros'] = st['n_zeros'] / float(nrows)
    # outliers (:222-223), thresholds in double, NaN counts as high (A.8)
    hi_t = q3 + k * (q3 - q1)
    lo_t = q1 - k * (q3 - q1)
    st['high_idx'] = int(np.sum(_spark_gt(vd, hi_t)))
    st['low_idx'] = int(np.sum(_spark_lt(vd, lo_t)))
    # histogram (:226 -> :38-63)
    edges, width = hist_edges(mn, mx, bins)
    counts = hist_counts(xs, edges)
    st['_hist'] = {'counts': counts, 'edges': edges, 'width': width}
    st['_thresholds'] = (hi_t, lo_t)
    return st


# ----------------------------------------------------------------------------
# categorical / constant / unique / date (describe.py:232-283)
# ----------------------------------------------------------------------------

def _py_values(arr, spark_t):
    """Row values as the driver sees them after toPandas (object array)."""
    if spark_t == 'date':
        return np.array(arr.cast(pa.date32()).to_pylist(), dtype=object)
    if spark_t == 'timestamp':
        return np.array([None if x is None else pd.Timestamp(x) for x in
                         arr.cast(pa.timestamp('us')).to_pylist()], dtype=object)
    return np.array(arr.to_pylist(), dtype=object)


def _nonnull_values(arr, spark_t):
    """`df.select(c).na.drop()` rows, in source order."""
    valid = _valid_mask(arr)
    if spark_t in ('float', 'double'):
        vals = _numeric_values(arr, spark_t)
        keep = valid & ~np.isnan(vals)
    else:
        keep = valid
    idx = np.nonzero(keep)[0]
    return idx


def _first_values_series(arr, spark_t, k):
    """`df.select(c).na.drop().limit(k).toPandas().ix[:, 0].value_counts()`
    (describe.py:276, :282)."""
    idx = _nonnull_values(arr, spark_t)[:k]
    sub = arr.take(pa.array(idx, pa.int64()))
    if spark_t in _INT_TYPES:
        col = pd.Series(np.asarray(sub.to_numpy(zero_copy_only=False)).astype(np.int64))
    elif spark_t in ('float', 'double'):
        col = pd.Series(np.asarray(sub.to_numpy(zero_copy_only=False)).astype(np.float64))
    elif spark_t == 'boolean':
        col = pd.Series(np.asarray(sub.to_numpy(zero_copy_only=False)).astype(bool))
    else:
        col = pd.Series(_py_values(sub, spark_t), dtype=object)
    return col.value_counts()


def _sort_key(v):
    if isinstance(v, (bytes, bytearray)):
        return bytes(v)
    return v


def _value_counts_fast(arr, spark_t, k=50):
    """(first k groups by (count desc, key asc), number of non-null rows,
    number of groups) through Arrow's hash aggregation (exact counts); only
    the groups at or above the k-th largest count are sorted by key."""
    import pyarrow.compute as pc
    a = arr.drop_null() if arr.null_count else arr
    if pa.types.is_dictionary(a.type):
        a = a.dictionary_decode()
    vc = pc.value_counts(a)
    keys = vc.field('values')
    cnt = np.asarray(vc.field('counts').to_numpy(zero_copy_only=False), dtype=np.int64)
    G = len(cnt)
    if G > k:
        thr = np.partition(cnt, G - k)[G - k]
        sel = np.nonzero(cnt >= thr)[0]
    else:
        sel = np.arange(G)
    sk = keys.take(pa.array(sel, pa.int64()))
    vals = _py_values(sk, spark_t).tolist()
    groups = sorted(zip(vals, cnt[sel].tolist()), key=lambda kv: (-kv[1], _sort_key(kv[0])))[:k]
    return groups, len(a), G


def categorical_stats(arr, spark_t, fast=False):
    """describe_categorical_1d (describe.py:250-271).  Group order: count desc,
    then key asc (the defined tie-break; the reference's orderBy is unstable)."""
    if fast:
        top50, nvals, ngroups = _value_counts_fast(arr, spark_t, 50)
        return _categorical_series(top50, nvals, ngroups)
    idx = _nonnull_values(arr, spark_t)
    vals = _py_values(arr.take(pa.array(idx, pa.int64())), spark_t)
    counts = {}
    for x in vals.tolist():
        counts[x] = counts.get(x, 0) + 1
    groups = sorted(counts.items(), key=lambda kv: (-kv[1], _sort_key(kv[0])))
    return _categorical_series(groups[:50], len(vals), len(groups))


def _categorical_series(top50, nvals, ngroups):
    groups = top50
    st = OrderedDict()
    st['top'] = groups[0][0]
    st['freq'] = np.int64(groups[0][1])
    top_keys = [g[0] for g in top50]
    top_counts = [g[1] for g in top50]
    others_count = nvals - sum(top_counts)
    others_distinct = ngroups - len(top50)
    vc = pd.Series(top_counts + [others_count, others_distinct],
                   index=pd.Index(top_keys + ['***Other Values***', '***Other Values Distinct Count***'],
                                  dtype=object),
                   dtype=np.int64)
    st['value_counts'] = vc
    st['type'] = 'CAT'
    return st


def date_stats(arr, spark_t, distinct_count, freq, fast=False):
    """describe_date_1d (describe.py:232-247)."""
    if fast:
        import pyarrow.compute as pc
        mm = pc.min_max(arr)
        vals = _py_values(pa.array([mm['min'].as_py(), mm['max'].as_py()], arr.type), spark_t)
    else:
        idx = _nonnull_values(arr, spark_t)
        vals = _py_values(arr.take(pa.array(idx, pa.int64())), spark_t)
    mn, mx = min(vals), max(vals)
    st = OrderedDict()
    if isinstance(mx, pd.Timestamp):
        st['min'] = str(mn.to_pydatetime())
        st['max'] = str(mx.to_pydatetime())
    else:
        st['min'] = mn
        st['max'] = mx
        st['range'] = mx - mn
    st['type'] = 'DATE'
    st['completeness_idx'] = float(distinct_count) / len(pd.date_range(start=st['min'], end=st['max'], freq=freq))
    return st


# ----------------------------------------------------------------------------
# describe_1d (describe.py:136-189)
# ----------------------------------------------------------------------------

def _distinct_count(arr, spark_t, fast=False):
    if fast and spark_t != 'null':
        return _distinct_count_fast(arr, spark_t)
    valid = _valid_mask(arr)
    if spark_t in _INT_TYPES:
        return int(np.unique(_numeric_values(arr, spark_t)[valid]).size)
    if spark_t in ('float', 'double'):
        return int(np.unique(_canon_float_keys(_numeric_values(arr, spark_t)[valid])).size)
    if spark_t == 'null':
        return 0
    vals = _py_values(arr, spark_t)[valid]
    return len(set(_sort_key(x) for x in vals.tolist()))


def _distinct_count_fast(arr, spark_t):
    """countDistinct: numeric keys by an in-place sort and a count of key
    changes, other types by Arrow's hash kernel -- the semantics of the exact
    count above."""
    valid = _valid_mask(arr)
    if spark_t in _INT_TYPES or spark_t in ('float', 'double'):
        v = _numeric_values(arr, spark_t)[valid]
        k = v if spark_t in _INT_TYPES else _canon_float_keys(v)
        k.sort()
        return int(k.size and 1 + np.count_nonzero(k[1:] != k[:-1]))
    import pyarrow.compute as pc
    a = arr.dictionary_decode() if pa.types.is_dictionary(arr.type) else arr
    return int(pc.count_distinct(a, mode='only_valid').as_py())


def describe_1d(arr, spark_t, nrows, bins, k, freq, raw, fast=False):
    if ('array' in spark_t) or ('struct' in spark_t) or ('map' in spark_t):
        raise NotImplementedError('Column {c} is of type {t} and cannot be analyzed'.format(c=raw['name'], t=spark_t))
    distinct = _distinct_count(arr, spark_t, fast)
    valid = _valid_mask(arr) if spark_t != 'null' else np.zeros(len(arr), bool)
    if spark_t in ('float', 'double'):
        cnt = int(np.sum(valid & ~np.isnan(_numeric_values(arr, spark_t))))
    else:
        cnt = int(valid.sum())
    res = OrderedDict()
    res['distinct_count'] = np.int64(distinct)
    res['count'] = np.int64(cnt)
    with np.errstate(all='ignore'):
        res['p_unique'] = np.float64(distinct) / float(cnt) if cnt else (
            np.float64('nan') if distinct == 0 else np.float64('inf'))
    res['is_unique'] = np.bool_(distinct == nrows)
    res['n_missing'] = np.int64(nrows - cnt)
    res['p_missing'] = np.float64(nrows - cnt) / float(nrows)
    res['p_infinite'] = np.int64(0)
    res['n_infinite'] = np.int64(0)
    res['memorysize'] = 0
    raw['distinct_count'] = distinct
    raw['count'] = cnt

    if distinct <= 1:
        st = OrderedDict([('type', 'CONST')])
        st['value_counts'] = (_first_values_series(arr, spark_t, 1) if spark_t != 'null'
                              else pd.Series([], dtype=object).value_counts())
    elif spark_t in _INT_TYPES or spark_t in ('float', 'double'):
        is_int = spark_t in _INT_TYPES
        st = numeric_stats(_numeric_values(arr, spark_t), valid, is_int, nrows, bins, k, fast)
        raw['hist'] = st.pop('_hist')
        raw['thresholds'] = st.pop('_thresholds')
        st['histogram'] = None            # filled by the caller (PNG renderer or None)
        st['mini_histogram'] = None
    elif spark_t in _DATE_TYPES:
        st = date_stats(arr, spark_t, distinct, freq.upper(), fast)
    elif bool(res['is_unique']):
        st = OrderedDict([('type', 'UNIQUE')])
        st['value_counts'] = _first_values_series(arr, spark_t, 50)
    else:
        st = categorical_stats(arr, spark_t, fast)
    res.update(st)
    if res['type'] == 'CAT' and res['n_missing'] > 0:          # :169-170
        res['distinct_count'] += 1
    # mode (:174-187)
    if res['count'] > res['distinct_count'] > 1:
        res['mode'] = res['top'] if 'top' in res else 0
    else:
        if 'value_counts' in res:
            vc = res['value_counts']
            res['mode'] = vc.index[0] if len(vc) else 'MISSING'
        else:
            res['mode'] = 0
    raw['type'] = res['type']
    return res


# ----------------------------------------------------------------------------
# corr_matrix (utils.py:20-36) and describe (describe.py:66-133)
# ----------------------------------------------------------------------------

def corr_matrix(table, columns, fast=False):
    """Pearson on rows with no null/NaN in any of `columns` (utils.py:27-31)."""
    keep = np.ones(table.num_rows, bool)
    mats = []
    for c in columns:
        arr = _column(table, c)
        t = spark_type_of(arr.type)
        v = _numeric_values(arr, t).astype(np.float64)
        keep &= _valid_mask(arr) & ~np.isnan(v)
        mats.append(v)
    X = np.stack(mats, axis=1)[keep]
    n = X.shape[0]
    C = len(columns)
    out = np.full((C, C), np.nan)
    if n > 0:
        means = np.array([_sum(X[:, j], fast) / n for j in range(C)])
        Xc = X - means
        G = Xc.T @ Xc
        with np.errstate(all='ignore'):
            dg = np.sqrt(np.diag(G))
            out = G / np.outer(dg, dg)
    return pd.DataFrame(out, index=list(columns), columns=list(columns))


def describe(table, bins=10, corr_reject=0.9, plot=None, **kwargs):
    """describe.py:66-133 on a pyarrow.Table.  `plot(hist_frame) -> str` renders
    the histogram strings; None leaves the raw counts in `profile_raw`."""
    d, _ = _describe_with_raw(table, bins, corr_reject, plot, **kwargs)
    return d


def profile_raw(table, bins=10, corr_reject=0.9, **kwargs):
    """(describe dict, per-column raw values: hist counts/edges, thresholds, corr)."""
    return _describe_with_raw(table, bins, corr_reject, None, **kwargs)


def _describe_column(args):
    """describe_1d of one column (picklable unit of work for describe_fast's
    process pool)."""
    arr, t, n, bins, k, freq, name, fast = args
    raw = {'name': name, 'spark_type': t}
    s = describe_1d(arr, t, n, bins, k, freq, raw, fast)
    return s, raw


def _describe_with_raw(table, bins, corr_reject, plot, fast=False, pool=None, **kwargs):
    if isinstance(table, pa.RecordBatch):
        table = pa.Table.from_batches([table])
    if not isinstance(table, pa.Table):
        raise TypeError('df must be of type pyspark.sql.DataFrame')
    n = table.num_rows
    table_stats = {'n': n}
    if n == 0:
        raise ValueError('df cannot be empty')
    k_vals, t_freq = kwargs.get('k_vals') or {}, kwargs.get('t_freq') or {}
    ldesc = OrderedDict()
    raws = OrderedDict()
    jobs = []
    for name in table.column_names:
        arr = _column(table, name)
        jobs.append((arr, spark_type_of(arr.type), n, bins, k_vals.get(name, 2), t_freq.get(name, 'D'), name, fast))
    results = list(pool.map(_describe_column, jobs)) if pool is not None else [_describe_column(j) for j in jobs]
    for name, (s, raw) in zip(table.column_names, results):
        if 'histogram' in s and plot is not None:
            h = raw['hist']
            frame = pd.DataFrame({'bin_id': np.arange(len(h['counts'])), 'count': h['counts'],
                                  'left_edge': h['edges'], 'width': h['width']})
            s['histogram'] = plot(frame, 'complete')
            s['mini_histogram'] = plot(frame, 'mini')
        ldesc[name] = pd.Series(list(s.values()), index=list(s.keys()), name=name, dtype=object)
        raws[name] = raw

    corr = None
    if corr_reject is not None:
        computable = [c for c in ldesc if ldesc[c]['type'] == 'NUM']
        if len(computable) > 0:
            corr = corr_matrix(table, computable, fast)
            for x, corr_x in corr.iterrows():
                for y, cv in corr_x.items():
                    if x == y:
                        break
                    if cv >= corr_reject:
                        ldesc[x] = pd.Series(['CORR', y, cv], index=['type', 'correlation_var', 'correlation'],
                                             name=x, dtype=object)
    variable_stats = pd.DataFrame(ldesc)
    table_stats['nvar'] = len(table.column_names)
    nm = pd.to_numeric(variable_stats.loc['n_missing'], errors='coerce')
    table_stats['total_missing'] = float(nm.sum()) / (table_stats['n'] * table_stats['nvar'])
    hi = pd.to_numeric(variable_stats.loc['high_idx'], errors='coerce')     # KeyError w/o NUM (:108)
    lo = pd.to_numeric(variable_stats.loc['low_idx'], errors='coerce')
    ct = pd.to_numeric(variable_stats.loc['count'], errors='coerce')
    table_stats['accuracy_idx'] = 1 - ((hi + lo) / ct).mean(skipna=True)
    memsize = 0
    table_stats['memsize'] = fmt_bytesize(memsize)
    table_stats['recordsize'] = fmt_bytesize(memsize / table_stats['n'])
    table_stats.update({k: 0 for k in ('NUM', 'DATE', 'CONST', 'CAT', 'UNIQUE', 'CORR')})
    table_stats.update(dict(variable_stats.loc['type'].value_counts()))
    table_stats['REJECTED'] = table_stats['CONST'] + table_stats['CORR']
    freq_dict = {}
    for var in variable_stats:
        v = variable_stats[var].get('value_counts', None) if 'value_counts' in variable_stats.index else None
        if isinstance(v, pd.Series):
            freq_dict[var] = v
    if 'value_counts' in variable_stats.index:
        variable_stats = variable_stats.drop('value_counts')
    variables = variable_stats.T
    # integral NUM columns: their 'sum' is float(wrapped int64) (describe.py:200
    # Sum of a LongType, upcast at :209), an exact value tests/compare.py checks
    # with == rather than the fp64 tolerance
    variables.attrs['integral_num'] = tuple(
        name for name, raw in raws.items()
        if raw.get('spark_type') in _INT_TYPES and name in ldesc and ldesc[name].get('type') == 'NUM')
    out = {'table': table_stats, 'variables': variables, 'freq': freq_dict}
    return out, {'columns': raws, 'corr': corr}
