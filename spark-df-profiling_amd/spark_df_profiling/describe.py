"""describe(): the reference's statistics entry point, computed on MI355X.

Drop-in for /root/reference/spark_df_profiling/describe.py:66 -- same
signature, same {'table', 'variables', 'freq'} result, same per-type key sets
(SURVEY.md Appendix B), same quirks (Appendix C) and the same errors
(TypeError for an unsupported input, ValueError('df cannot be empty'),
NotImplementedError for array/struct/map columns).  The input widens from a
Spark DataFrame to Arrow: a pyarrow Table/RecordBatch, a Spark DataFrame
(collected as Arrow when pyspark is present) or a DeviceTable already in HBM.

All row-level work runs in libsdp.so (engine.py); this module only performs the
driver-side assembly the reference performs in pandas.
"""

from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np
import pandas as pd
import pyarrow as pa

from . import _native as nat
from .columns import DATE_TYPES, FLOAT_TYPES, INT_TYPES, DeviceColumn, DeviceTable
from .engine import PROBS, TOPK, Engine, hist_edges  # noqa: F401
from .utils import corr_from_gram, pretty_name

OTHER_VALUES = '***Other Values***'                           # describe.py:262
OTHER_DISTINCT = '***Other Values Distinct Count***'          # describe.py:263
# sharded runs: the first all-gather round's room for one column's two
# rendered histograms (base64 PNG strings, 25-28 KB pickled per column on
# normal / lognormal / t3 / uniform data), so the images exchange needs no
# second round (an overflow only costs that round)
IMAGE_CAP_PER_COLUMN = 48 * 1024


def fmt_bytesize(num, suffix='B'):
    """Human-readable byte size, as the reference's formatters.fmt_bytesize."""
    units = ['', 'Ki', 'Mi', 'Gi', 'Ti', 'Pi', 'Ei', 'Zi']
    for u in units:
        if abs(num) < 1024.0:
            return "%3.1f %s%s" % (num, u, suffix)
        num /= 1024.0
    return "%.1f %s%s" % (num, 'Yi', suffix)


def as_device_table(df, device=None) -> DeviceTable:
    if isinstance(df, DeviceTable):
        return df
    if isinstance(df, (pa.Table, pa.RecordBatch)):
        return DeviceTable.from_arrow(df, device)
    import os
    if isinstance(df, (str, os.PathLike)) and str(df).endswith('.parquet'):
        # the reference's inputs come from spark.read.parquet (examples/Demo.ipynb:63)
        return DeviceTable.from_parquet(str(df), device=device)
    if type(df).__module__.startswith('pyspark'):
        return spark_to_device(df, device)
    batches = _batch_stream(df)
    if batches is not None:
        from . import ingest
        schema, it, rows = batches
        return ingest.stream_batches(schema, rows, it, device)
    raise TypeError('df must be of type pyspark.sql.DataFrame, pyarrow.Table, a .parquet path or DeviceTable')


def _batch_stream(obj):
    """(schema, batch iterable, rows or None) of an Arrow RecordBatchReader, a
    list of RecordBatches or an iterator yielding them; None for anything else."""
    import itertools
    if isinstance(obj, pa.RecordBatchReader):
        return obj.schema, obj, None
    if isinstance(obj, (list, tuple)):
        if obj and all(isinstance(b, pa.RecordBatch) for b in obj):
            return obj[0].schema, obj, sum(b.num_rows for b in obj)
        return None
    if hasattr(obj, '__next__') and hasattr(obj, '__iter__'):
        first = next(obj, None)
        if not isinstance(first, pa.RecordBatch):
            return None
        return first.schema, itertools.chain([first], obj), None
    return None


def spark_batches(df):
    """A Spark DataFrame (pyspark is optional: only its duck type is used) as
    Arrow RecordBatches for the staging pipeline, never row by row -- the
    counterpart of the reference's per-statistic Spark jobs (describe.py:71-283)
    is one columnar transfer followed by HBM-resident passes.  Returns
    (schema or None, batches, rows or None):
      Spark >= 4.0   df.toArrow()                  -> the Table's batches
      Spark 2.3-3.x  df._collect_as_arrow()        -> its batches (a list, or an
                                                      iterator: streamed as they come)
      otherwise      df.toPandas() (Arrow-accelerated when
                     spark.sql.execution.arrow.enabled)"""
    to_arrow = getattr(df, 'toArrow', None)
    if to_arrow is not None:
        t = to_arrow()
        return t.schema, t.to_batches(), t.num_rows
    collect = getattr(df, '_collect_as_arrow', None)
    if collect is not None:
        got = collect()
        if isinstance(got, pa.Table):
            return got.schema, got.to_batches(), got.num_rows
        st = _batch_stream(got if isinstance(got, (list, tuple)) else iter(got))
        if st is None:
            if isinstance(got, (list, tuple)) and not got:
                return None, [], 0
            raise TypeError('_collect_as_arrow() did not yield pyarrow RecordBatches')
        return st
    to_pandas = getattr(df, 'toPandas', None)
    if to_pandas is None:
        raise TypeError('Spark DataFrame without toArrow/_collect_as_arrow/toPandas')
    t = pa.Table.from_pandas(to_pandas(), preserve_index=False)
    return t.schema, t.to_batches(), t.num_rows


def spark_to_arrow(df):
    """spark_batches collected into one Arrow Table (host)."""
    schema, batches, _ = spark_batches(df)
    batches = list(batches)
    if schema is None:
        return pa.table({})
    return pa.Table.from_batches(batches, schema=schema)


_SPARK_KIND = {'tinyint': 'fixed', 'smallint': 'fixed', 'int': 'fixed', 'bigint': 'fixed', 'float': 'fixed',
               'double': 'fixed', 'boolean': 'fixed', 'date': 'fixed', 'timestamp': 'fixed',
               'string': 'bytes', 'binary': 'bytes'}


def apply_spark_dtypes(table: DeviceTable, dtypes):
    """Dispatch by Spark's own type strings (`df.dtypes`, describe.py:137) where
    the DataFrame provides them: the column's spark_type becomes Spark's string
    (e.g. 'decimal(10,2)', which describe.py:158-164 sends to CAT/UNIQUE).  A
    string of another storage kind than the transferred Arrow column is
    rejected (the transfer does not match the DataFrame)."""
    for col in table.columns:
        st = dtypes.get(col.name)
        if st is None or st == col.spark_type:
            continue
        kind = 'bytes' if st.startswith('decimal') else _SPARK_KIND.get(st)
        if kind is not None and col.kind not in (kind, 'null'):
            raise TypeError('column %s: Spark type %s but the Arrow transfer holds %s' % (col.name, st,
                                                                                   col.spark_type))
        col.spark_type = st
    return table


def spark_to_device(df, device=None) -> DeviceTable:
    """A Spark DataFrame straight into HBM: its Arrow batches go through the
    pinned double-buffered staging pipeline (ingest.stream_batches) as they
    arrive -- a batch iterator is never concatenated on the host -- and the
    column types dispatch by `df.dtypes` (describe.py:137)."""
    from . import ingest
    rows_hint = None
    count = getattr(df, 'count', None)
    schema, batches, rows = spark_batches(df)
    if rows is None and callable(count):
        rows_hint = int(count())                  # the reference's n = df.count() (describe.py:71)
    if schema is None:
        raise ValueError('df cannot be empty')
    table = ingest.stream_batches(schema, rows, batches, device, rows_hint=rows_hint)
    dtypes = getattr(df, 'dtypes', None)
    if dtypes:
        apply_spark_dtypes(table, dict(dtypes))
    return table


def _series(values, col: DeviceColumn) -> pd.Series:
    """The one-column pandas frame `toPandas().ix[:, 0]` yields for `values`."""
    st = col.spark_type
    if st in INT_TYPES:
        return pd.Series(np.asarray(values, dtype=np.int64))
    if st in ('float', 'double'):
        return pd.Series(np.asarray(values, dtype=np.float64))
    if st == 'boolean':
        return pd.Series(np.asarray(values, dtype=bool))
    if st == 'timestamp':
        return pd.Series(pd.to_datetime(list(values)) if len(values) else pd.Series([], dtype='datetime64[ns]'))
    return pd.Series(list(values), dtype=object)


def _value_counts_first(engine, col, k):
    """`df.select(c).na.drop().limit(k).toPandas().ix[:, 0].value_counts()`
    (describe.py:276, :282) -- the rows are found on the GPU."""
    return _series(engine.first_rows(col, k), col).value_counts()


def _distinct_hint(p1, spark_t):
    """Upper bound of a NUM column's distinct count from pass 1: the valid
    rows, or the integral value range."""
    hint = p1['n_valid']
    if spark_t in INT_TYPES and p1['count']:
        hint = min(hint, p1['imax'] - p1['imin'] + 1 + (p1['n_valid'] - p1['count']))
    return hint


def _distinct_count(engine, col, p1, hint):
    """countDistinct (describe.py:143) of a NUM/DATE column: a value bitmap when
    the integral range from pass 1 is small, else exact hash grouping."""
    if (p1['count'] and col.kind == 'fixed' and col.dtype in engine.BITMAP_DTYPES
            and p1['imax'] - p1['imin'] + 1 <= nat.BITMAP_MAX_BITS):
        return engine.distinct_bitmap(col, p1['imin'], p1['imax'] - p1['imin'] + 1)
    return engine.distinct_fixed(col, with_counts=False, capacity_hint=hint)['groups']


def describe_1d(engine: Engine, col: DeviceColumn, nrows, bins, k, freq, bundle):
    """describe.py:136-189 for one column; `bundle` receives raw engine outputs."""
    spark_t = col.spark_type
    if ('array' in spark_t) or ('struct' in spark_t) or ('map' in spark_t) or col.kind == 'nested':
        raise NotImplementedError('Column {c} is of type {t} and cannot be analyzed'.format(c=col.name, t=spark_t))

    numeric = spark_t in INT_TYPES or spark_t in ('float', 'double')
    tab = None
    p1_pack = None
    if col.kind == 'null':
        distinct, count = 0, 0
    elif numeric:
        p1_pack = bundle.pop('p1_pack', None) or engine.numeric_pass1(col)
        p1 = p1_pack[0]
        bundle['p1'] = p1
        count = p1['count']
        distinct = bundle.pop('distinct_pre', None)
        if distinct is None:
            distinct = _distinct_count(engine, col, p1, _distinct_hint(p1, spark_t))
    elif spark_t in DATE_TYPES:
        p1 = bundle.pop('minmax_pre', None) or engine.minmax_pass(col)
        bundle['minmax'] = p1
        count = p1['count']
        distinct = bundle.pop('distinct_pre', None)
        if distinct is None:
            hint = p1['n_valid']
            if p1['count']:
                hint = min(hint, p1['imax'] - p1['imin'] + 1)
            distinct = _distinct_count(engine, col, p1, hint)
    elif col.kind == 'fixed':                      # boolean, decimal(20,0) from uint64
        tab = engine.distinct_fixed(col, with_counts=True)
        distinct, count = tab['groups'], tab['rows']
    else:                                          # string, binary, decimal
        tab = bundle.pop('tab_pre', None) or engine.value_counts_bytes(col)
        distinct, count = tab['groups'], tab['rows']

    res = OrderedDict()
    res['distinct_count'] = np.int64(distinct)
    res['count'] = np.int64(count)
    with np.errstate(divide='ignore', invalid='ignore'):
        res['p_unique'] = np.float64(distinct) / np.float64(count)
    res['is_unique'] = np.bool_(distinct == nrows)
    res['n_missing'] = np.int64(nrows - count)
    res['p_missing'] = np.float64(nrows - count) / float(nrows)
    res['p_infinite'] = np.int64(0)
    res['n_infinite'] = np.int64(0)
    res['memorysize'] = 0
    bundle.update({'distinct_count': int(distinct), 'count': int(count)})

    if distinct <= 1:
        stats = OrderedDict([('type', 'CONST')])
        stats['value_counts'] = _value_counts_first(engine, col, 1)
    elif numeric:
        st = bundle.pop('numeric_pre', None)
        if st is None:
            st = engine.numeric_stats(col, bins=bins, k=k, p1_pack=p1_pack)
        elif st.error is not None:
            raise st.error                     # e.g. describe.py:46 with bins=1
        bundle['numeric'] = st
        stats = _numeric_series(st, nrows)
    elif spark_t in DATE_TYPES:
        stats = _date_series(engine, col, bundle['minmax'], distinct, freq.upper())
    elif bool(res['is_unique']):
        stats = OrderedDict([('type', 'UNIQUE')])
        stats['value_counts'] = _value_counts_first(engine, col, 50)
    else:
        stats = _categorical_series(engine, col, tab, count, bundle)
    res.update(stats)
    if res['type'] == 'CAT' and res['n_missing'] > 0:           # describe.py:169-170
        res['distinct_count'] += 1
    # mode (describe.py:174-187)
    if res['count'] > res['distinct_count'] > 1:
        res['mode'] = res['top'] if 'top' in res else 0
    elif 'value_counts' in res:
        vc = res['value_counts']
        res['mode'] = vc.index[0] if len(vc) else 'MISSING'
    else:
        res['mode'] = 0
    return res


def _const_numeric(st):
    """describe_1d's CONST test (distinct <= 1, describe.py:156) from pass-1
    alone: no non-null value, or one value and no NaN (NaN is a distinct
    value of its own for countDistinct)."""
    return st.count == 0 or (st.min == st.max and st.n_nan == 0)


def _is_numeric(col):
    st = col.spark_type
    nested = ('array' in st) or ('struct' in st) or ('map' in st) or col.kind == 'nested'
    return col.kind != 'null' and not nested and (st in INT_TYPES or st in ('float', 'double'))


def _is_date(col):
    """describe_date_1d's columns (describe.py:162, :232): fixed-width date/timestamp."""
    return col.kind == 'fixed' and col.spark_type in DATE_TYPES


def _is_byte_keyed(col):
    """describe_1d's string/binary/decimal branch (value counts on byte keys)."""
    st = col.spark_type
    nested = ('array' in st) or ('struct' in st) or ('map' in st) or col.kind == 'nested'
    return (col.kind == 'bytes' and not nested and st not in INT_TYPES and st not in ('float', 'double')
            and st not in DATE_TYPES)


def _numeric_series(st, nrows):
    """Key order and scalar types of describe_numeric_1d (describe.py:193-229)."""
    s = OrderedDict()
    for key in ('mean', 'min', 'max', 'variance', 'kurtosis', 'std', 'skewness', 'sum'):
        s[key] = np.float64(getattr(st, key))
    for p in PROBS:
        s[pretty_name(p)] = np.float64(st.quantiles[p])
    with np.errstate(all='ignore'):
        s['range'] = np.float64(st.max) - np.float64(st.min)
        q3, q1 = s[pretty_name(0.75)], s[pretty_name(0.25)]
        s['iqr'] = q3 - q1
        s['cv'] = s['std'] / float(s['mean'])
        s['mad'] = np.float64(st.mad) / float(st.count)
    s['type'] = 'NUM'
    s['n_zeros'] = int(st.n_zero)
    s['p_zeros'] = st.n_zero / float(nrows)
    s['high_idx'] = int(st.high_idx)
    s['low_idx'] = int(st.low_idx)
    s['histogram'] = None            # filled after the GPU work (PNG rendering, plot.py)
    s['mini_histogram'] = None
    return s


def _date_series(engine, col, p1, distinct, freq):
    """describe_date_1d (describe.py:232-247)."""
    from .engine import host_value
    mn = host_value(p1['imin'], col)
    mx = host_value(p1['imax'], col)
    s = OrderedDict()
    if isinstance(mx, pd.Timestamp):
        s['min'] = str(mn.to_pydatetime())
        s['max'] = str(mx.to_pydatetime())
    else:
        s['min'] = mn
        s['max'] = mx
        s['range'] = mx - mn
    s['type'] = 'DATE'
    s['completeness_idx'] = float(distinct) / len(pd.date_range(start=s['min'], end=s['max'], freq=freq))
    return s


def _categorical_series(engine, col, tab, count, bundle):
    """describe_categorical_1d (describe.py:250-271).  Groups ordered by count
    desc then key asc (the reference's orderBy leaves ties unspecified)."""
    pairs = bundle.pop('topk_pre', None)
    if pairs is None:
        pairs = engine.global_topk(tab, col, TOPK)
    values = [v for v, _ in pairs]
    counts = [int(c) for _, c in pairs]
    bundle['topk'] = pairs
    groups = tab['groups']
    s = OrderedDict()
    s['top'] = values[0]
    s['freq'] = np.int64(counts[0])
    others_count = int(count) - sum(counts)
    others_distinct = int(groups) - len(counts)
    s['value_counts'] = pd.Series(counts + [others_count, others_distinct],
                                  index=pd.Index(values + [OTHER_VALUES, OTHER_DISTINCT], dtype=object),
                                  dtype=np.int64)
    s['type'] = 'CAT'
    return s


def describe(df, bins=10, corr_reject=0.9, **kwargs):
    """describe.py:66-133.  Extra keyword arguments beyond the reference's
    (k_vals, t_freq): ``comm`` (a comm.TorchComm for a row-sharded table -- each
    rank passes its own row range), ``device``, ``plots`` (default True:
    histogram PNGs as the reference stores them) and ``raw`` (a dict that
    receives the per-column engine outputs, e.g. exact histogram counts),
    ``quantile_mode`` ('exact', the default: float quantiles are the element at
    rank ceil(pN), inside percentile_approx's rank window; 'gk': Spark 2.x's
    percentile_approx element for ``spark_partitions`` contiguous partitions
    (default: one per rank), restated from QuantileSummaries; on a sharded
    table each rank's rows form spark_partitions / world of them)."""
    comm = kwargs.pop('comm', None)
    device = kwargs.pop('device', None)
    plots = kwargs.pop('plots', True)
    raw = kwargs.pop('raw', None)
    quantile_mode = kwargs.pop('quantile_mode', 'exact')
    if quantile_mode not in ('exact', 'gk'):
        raise ValueError("quantile_mode must be 'exact' or 'gk'")
    partitions = kwargs.pop('spark_partitions', None)
    accuracy = int(kwargs.pop('accuracy', 10000))
    table = as_device_table(df, device)
    engine = Engine(device=device, comm=comm)
    gk = None
    if quantile_mode == 'gk':
        # default: one Spark partition per rank; a sharded table's partitions
        # are split evenly over the ranks (rank r holds k consecutive ones)
        w = engine.comm.world
        partitions = int(partitions) if partitions is not None else w
        if partitions < 1 or partitions % w:
            raise ValueError('spark_partitions (%d) must be a positive multiple of the number of ranks (%d)'
                             % (partitions, w))
        gk = {'partitions': partitions, 'accuracy': accuracy}
    import torch
    n_local = table.num_rows
    n = int(engine.comm.allreduce_sum(torch.full((1,), n_local, dtype=torch.int64, device=engine.device)).item())
    table_stats = {'n': n}
    if n == 0:
        raise ValueError('df cannot be empty')

    k_vals, t_freq = kwargs.get('k_vals') or {}, kwargs.get('t_freq') or {}
    bundles = OrderedDict((col.name, {'spark_type': col.spark_type}) for col in table.columns)
    ldesc = OrderedDict((col.name, None) for col in table.columns)
    pending = OrderedDict()

    world, rank, sharded = engine.comm.world, engine.comm.rank, engine.comm.sharded
    owner = {col.name: i % world for i, col in enumerate(table.columns)}

    early_plots = {}

    def one(eng, col):
        res = describe_1d(eng, col, n, bins, k_vals.get(col.name, 2), t_freq.get(col.name, 'D'), bundles[col.name])
        # rendered by worker processes while the next columns' kernels run; on
        # a sharded table each rank renders the columns it owns (index % world)
        mine = owner[col.name] == rank
        fut = early_plots.pop(col.name, None)
        if fut is None and plots and res['type'] == 'NUM' and mine:
            fut = _submit_plot(bundles[col.name]['numeric'])
        if res['type'] != 'NUM':
            fut = None
        return res, fut

    workers = column_workers(engine, kwargs.pop('workers', None))
    if gk is not None:
        workers = 1                      # the GK quantiles ride the whole-table numeric stage
    if workers == 1:
        # whole-table stages: pass 1 of every numeric column (two readbacks),
        # then every column's order statistics and pass 2 (two more) -- the
        # per-column loop below only counts distincts and assembles
        num_cols = [c for c in table.columns if _is_numeric(c)]
        # date / timestamp columns: min/max in the numeric pass-1 launches and readback
        date_cols = [c for c in table.columns if _is_date(c)]
        # byte columns: their heavy-key samples ride the same readback
        byte_cols = [c for c in table.columns if _is_byte_keyed(c)]
        packs, date_p1 = engine.numeric_pass1_batch(num_cols, minmax_cols=date_cols, byte_cols=byte_cols) \
            if date_cols else (engine.numeric_pass1_batch(num_cols, byte_cols=byte_cols), [])
        for col, p1 in zip(date_cols, date_p1):
            bundles[col.name]['minmax_pre'] = p1
        p1s = [pk[0] for pk in packs]
        hints = [_distinct_hint(p1, c.spark_type) for c, p1 in zip(num_cols, p1s)]
        bounds = [(p1['imin'], p1['imax']) if p1['count'] else None for p1 in p1s]
        # columns whose countDistinct partitions by hash: pass 2 also counts
        # their level-1 buckets (one column read fewer)
        # (a column found sorted in pass 1 already has its count: sdp_sorted_distinct)
        known = [p1.get('sorted_distinct') for p1 in p1s]
        # (date columns join the distinct batch: their distinct hint is the day range)
        dcols = num_cols + date_cols
        dhints = hints + [min(p1['n_valid'], p1['imax'] - p1['imin'] + 1) if p1['count'] else p1['n_valid']
                          for p1 in date_p1]
        dbounds = bounds + [(p1['imin'], p1['imax']) if p1['count'] else None for p1 in date_p1]
        dknown = known + [None] * len(date_cols)
        # every column's distinct path is chosen ONCE, here, before pass 2 and
        # the grouping consume the pass-1 heavy-key samples it depends on; pass 2's
        # pre-counts and the distinct batch both follow it
        dpaths = engine.distinct_paths_sharded(dcols, dhints, dbounds, n) if sharded else \
            engine.distinct_paths(dcols, dhints, dbounds)
        paths = dpaths[:len(num_cols)]
        group_cols = {i for i, pth in enumerate(paths) if pth == 'group' and known[i] is None}
        # 32-bit key spaces (sdp_distinct32): pass 2 takes their level-1 count too
        count32_cols = {i: (bounds[i][0] if bounds[i] is not None else 0)
                        for i, pth in enumerate(paths) if pth == 'bits32' and known[i] is None}
        stats = engine.numeric_stats_batch(num_cols, packs, bins, [k_vals.get(c.name, 2) for c in num_cols],
                                           group_cols=group_cols, gk=gk, count32_cols=count32_cols)
        to_plot = []
        for col, pack, st in zip(num_cols, packs, stats):
            bundles[col.name]['p1_pack'] = pack
            if st is not None:
                bundles[col.name]['numeric_pre'] = st
                # the histogram images render while the distinct counts run; a
                # column that turns out CONST (one distinct value) is never NUM
                if plots and st.error is None and owner[col.name] == rank and not _const_numeric(st):
                    to_plot.append((col.name, st))
        early_plots.update(zip([name for name, _ in to_plot], _submit_plots([st for _, st in to_plot])))
        # every NUM column's countDistinct with shared readbacks (and, sharded,
        # shared collectives), on the paths chosen above
        dist = engine.distinct_batch(dcols, dhints, dbounds, dknown, paths=dpaths) if not sharded else \
            engine.distinct_batch_sharded(dcols, dhints, dbounds, dknown, n_all=n, paths=dpaths)
        for col, d in zip(dcols, dist):
            bundles[col.name]['distinct_pre'] = d
        # every string/binary/decimal column's value counts with shared
        # readbacks (sharded: then each column's owner exchange, in column order)
        cat_items = []
        for col, tab in zip(byte_cols, engine.value_counts_bytes_batch(byte_cols)):
            bundles[col.name]['tab_pre'] = tab
            if 1 < tab['groups'] != n:                 # CAT (describe.py:163-168): its top-50 is needed
                cat_items.append((col, tab))
        # every CAT column's top-50 and their values with shared readbacks
        for (col, tab), pairs in zip(cat_items, engine.global_topk_batch([(t, c) for c, t in cat_items], TOPK)):
            bundles[col.name]['topk_pre'] = pairs
    if workers > 1:
        done = _describe_concurrent(engine, table.columns, one, workers)
    else:
        done = {col.name: one(engine, col) for col in table.columns}
    for name in ldesc:
        ldesc[name], fut = done[name]
        if fut is not None:
            pending[name] = fut

    images = {name: (fut.result() if hasattr(fut, 'result') else fut) for name, fut in pending.items()}
    if plots and sharded:
        # one exchange of the rendered strings (~28 KB per NUM column),
        # in one round: the cap every rank derives from the same count of
        # plotted (NUM) columns -- the types come from global statistics
        n_plot = sum(1 for d in ldesc.values() if d['type'] == 'NUM')
        for part in engine.comm.allgather_object(images, cap=IMAGE_CAP_PER_COLUMN * max(1, n_plot)):
            images.update(part)
    for name, (hist, mini) in images.items():
        ldesc[name]['histogram'], ldesc[name]['mini_histogram'] = hist, mini

    # correlation rejection (describe.py:89-100)
    corr = None
    if corr_reject is not None:
        computable = [c for c in ldesc if ldesc[c]['type'] == 'NUM']
        if len(computable) > 0:
            corr = corr_matrix(engine, table, computable, bundles)
            for x, corr_x in corr.iterrows():
                for y, cv in corr_x.items():
                    if x == y:
                        break
                    if cv >= corr_reject:
                        ldesc[x] = OrderedDict([('type', 'CORR'), ('correlation_var', y), ('correlation', cv)])
    if raw is not None:
        raw.update({'columns': bundles, 'corr': corr})
    return _assemble(ldesc, table_stats, len(table.columns))


def column_workers(engine, requested=None):
    """Columns profiled at once on one device (SDP_COLUMN_WORKERS, default 1).
    Each worker owns a HIP stream, so one column's latency-bound grouping
    kernels overlap another's VALU-bound moment passes and the host-side
    readbacks of both.  Sharded runs stay sequential: every rank must issue
    its collectives in the same order."""
    import os
    w = requested if requested is not None else int(os.environ.get('SDP_COLUMN_WORKERS', '1'))
    if engine.comm.sharded or engine.device.type != 'cuda':
        return 1
    return max(1, int(w))


def _column_temp_bytes(col):
    """Peak device temporaries of one column's profile: the grouping record
    buffers (two generations) plus (key, count) outputs where counts are kept."""
    n = col.length
    if col.kind == 'bytes':
        return 64 * n
    if col.kind == 'fixed':
        numeric = col.spark_type in INT_TYPES or col.spark_type in ('float', 'double')
        return (16 if numeric else 32) * n
    return 0


class _DeviceBudget:
    """Admits a column only while the temporaries of the columns in flight
    fit the device memory left after the resident table."""

    def __init__(self, device, reserve=4 << 30):
        import threading
        import torch
        free, _ = torch.cuda.mem_get_info(device)
        self.cap = max(0, free - reserve)
        self.used = 0
        self.busy = 0
        self.cv = threading.Condition()

    def acquire(self, need):
        with self.cv:
            # a column larger than the whole budget runs alone
            self.cv.wait_for(lambda: self.busy == 0 or self.used + need <= self.cap)
            self.used += need
            self.busy += 1

    def release(self, need):
        with self.cv:
            self.used -= need
            self.busy -= 1
            self.cv.notify_all()


def _describe_concurrent(engine, columns, one, workers):
    """Run `one(engine, col)` for every column on `workers` threads, each with
    its own stream and Engine; largest columns first.  Results are per column
    and independent of the schedule."""
    import threading
    import torch
    from concurrent.futures import ThreadPoolExecutor
    dev = engine.device
    torch.cuda.synchronize(dev)             # the table's uploads are visible to every stream
    budget = _DeviceBudget(dev)
    local = threading.local()

    def task(col):
        if not hasattr(local, 'engine'):
            local.stream = torch.cuda.Stream(device=dev)
            local.engine = Engine(device=dev, comm=engine.comm, stream=local.stream)
        need = _column_temp_bytes(col)
        budget.acquire(need)
        try:
            with torch.cuda.stream(local.stream):
                out = one(local.engine, col)
            local.stream.synchronize()
        finally:
            budget.release(need)
        return out

    order = sorted(columns, key=lambda c: -_column_temp_bytes(c))
    with ThreadPoolExecutor(max_workers=workers, thread_name_prefix='sdp-col') as ex:
        futs = {col.name: ex.submit(task, col) for col in order}
        return {name: f.result() for name, f in futs.items()}


def _submit_plot(st):
    """describe.py:227-228 histogram + mini_histogram for one NUM column: a
    pool future, or the strings themselves when SDP_PLOT_WORKERS=0."""
    return _submit_plots([st])[0]


def _submit_plots(sts):
    """_submit_plot of many columns, grouped into a few pool tasks."""
    from . import plot
    import os
    if os.environ.get('SDP_PLOT_WORKERS', '') == '0':
        return [plot.render_pair(st.hist_counts, st.edges, st.width) for st in sts]
    return plot.submit_batch([(st.hist_counts, st.edges, st.width) for st in sts])


def corr_matrix(engine, table, columns, bundles):
    """utils.py:20-36 on the GPU: one listwise-deletion mask + one Gram product."""
    cols = [table.column(c) for c in columns]
    shifts = [bundles[c]['numeric'].mean for c in columns]
    check_nan = [bundles[c]['numeric'].n_nan > 0 for c in columns]
    G, s, nk = engine.gram(cols, shifts, check_nan)
    rho = corr_from_gram(G, s, nk)
    return pd.DataFrame(rho, index=list(columns), columns=list(columns))


def _stats_frame(ldesc):
    """pd.DataFrame({name: pd.Series(stats, dtype=object)}) (describe.py:102)
    built in one piece: pandas aligns the columns' key sets to their union,
    which is taken from one column per distinct key set (a 512-column table has
    a handful), and the object matrix is filled directly -- 512 Series
    alignments took ~60 ms."""
    if not ldesc:
        return pd.DataFrame({})
    reps = {}
    for k, v in ldesc.items():
        reps.setdefault(tuple(v.keys()), k)
    index = pd.DataFrame({k: pd.Series([None] * len(keys), index=list(keys), name=k, dtype=object)
                          for keys, k in reps.items()}).index
    pos = {key: i for i, key in enumerate(index)}
    arr = np.empty((len(index), len(ldesc)), dtype=object)
    arr[:] = np.nan
    for j, v in enumerate(ldesc.values()):
        for key, val in v.items():
            arr[pos[key], j] = val
    return pd.DataFrame(arr, index=index, columns=list(ldesc.keys()), dtype=object)


def _assemble(ldesc, table_stats, nvar):
    """describe.py:102-133."""
    variable_stats = _stats_frame(ldesc)
    table_stats['nvar'] = nvar
    n = table_stats['n']
    n_missing = pd.to_numeric(variable_stats.loc['n_missing'], errors='coerce')
    table_stats['total_missing'] = float(n_missing.sum()) / (n * nvar)
    high = pd.to_numeric(variable_stats.loc['high_idx'], errors='coerce')     # KeyError without NUM (:108)
    low = pd.to_numeric(variable_stats.loc['low_idx'], errors='coerce')
    cnt = pd.to_numeric(variable_stats.loc['count'], errors='coerce')
    table_stats['accuracy_idx'] = 1 - ((high + low) / cnt).mean(skipna=True)
    memsize = 0
    table_stats['memsize'] = fmt_bytesize(memsize)
    table_stats['recordsize'] = fmt_bytesize(memsize / n)
    table_stats.update({k: 0 for k in ('NUM', 'DATE', 'CONST', 'CAT', 'UNIQUE', 'CORR')})
    table_stats.update(dict(variable_stats.loc['type'].value_counts()))
    table_stats['REJECTED'] = table_stats['CONST'] + table_stats['CORR']
    freq_dict = {}
    if 'value_counts' in variable_stats.index:
        for var in variable_stats:
            v = variable_stats[var]['value_counts']
            if isinstance(v, pd.Series):
                freq_dict[var] = v
        variable_stats = variable_stats.drop('value_counts')
    return {'table': table_stats, 'variables': variable_stats.T, 'freq': freq_dict}
