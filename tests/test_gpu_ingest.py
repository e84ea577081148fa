"""Arrow / Parquet staging pipeline (ingest.py): the
streamed upload must produce the same Arrow-layout device buffers -- and so the
same describe() -- as the whole-column upload, for every column type, odd
chunk sizes (bitmaps not byte aligned), nulls, NaN, long strings and the
types that fall back to the whole-column path -- and describe() of the
streamed and the parquet-loaded tables equals the oracle's on the host table."""

import decimal

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from compare import assert_describe_equal

pytestmark = pytest.mark.gpu


def _table(n=9000, seed=7):
    g = np.random.default_rng(seed)
    mask = g.random(n) < 0.07
    f = g.standard_normal(n)
    f[g.random(n) < 0.01] = np.nan
    words = np.array(['a', 'bb', 'ccc', 'dddd', 'x' * 15, 'y' * 16, 'z' * 17, 'long-' * 9, ''], dtype=object)
    s = words[g.integers(0, len(words), n)]
    cols = {
        'f64': pa.array(f, mask=mask),
        'i64': pa.array(g.integers(-10 ** 12, 10 ** 12, n)),
        'i32': pa.array(g.integers(0, 50, n).astype(np.int32), mask=g.random(n) < 0.3),
        'f32': pa.array(g.random(n).astype(np.float32)),
        'flag': pa.array(g.random(n) < 0.4, mask=g.random(n) < 0.1),
        'day': pa.array((g.integers(0, 20000, n)).astype(np.int32), type=pa.date32()),
        'ts': pa.array(g.integers(0, 10 ** 15, n), type=pa.timestamp('us')),
        'word': pa.array(list(s), mask=g.random(n) < 0.05, type=pa.string()),
        'lword': pa.array(list(s), type=pa.large_string()),
        'blob': pa.array([x.encode() for x in s], type=pa.binary()),
        'dec': pa.array([decimal.Decimal(int(v)).scaleb(-2) for v in g.integers(-10 ** 6, 10 ** 6, n)],
                        type=pa.decimal128(12, 2)),
        'none': pa.nulls(n),
    }
    return pa.table(cols)


def _rechunk(tab, sizes):
    out, start = [], 0
    while start < tab.num_rows:
        for m in sizes:
            if start >= tab.num_rows:
                break
            out.append(tab.slice(start, m))
            start += m
    return pa.concat_tables(out)


def _bits(t, off, n):
    b = t.cpu().numpy()
    return np.unpackbits(b, bitorder='little')[off:off + n]


def _assert_same_buffers(a, b):
    for ca, cb in zip(a.columns, b.columns):
        assert (ca.name, ca.kind, ca.dtype, ca.length) == (cb.name, cb.kind, cb.dtype, cb.length), ca.name
        n = ca.length
        va = _bits(ca.validity, ca.bit_offset, n) if ca.validity is not None else np.ones(n, np.uint8)
        vb = _bits(cb.validity, cb.bit_offset, n) if cb.validity is not None else np.ones(n, np.uint8)
        assert np.array_equal(va, vb), ca.name
        ok = va.astype(bool)
        if ca.kind == 'fixed' and ca.values is not None:
            from spark_df_profiling import _native as nat
            if ca.dtype == nat.BOOL:
                assert np.array_equal(_bits(ca.values, ca.bit_offset, n)[ok], _bits(cb.values, cb.bit_offset, n)[ok])
            else:
                xa, xb = ca.values.cpu().numpy()[:n], cb.values.cpu().numpy()[:n]
                assert np.array_equal(xa[ok].view(np.uint8), xb[ok].view(np.uint8)), ca.name
        elif ca.kind == 'bytes' and not ca.fixed_width:
            oa = ca.offsets.cpu().numpy().astype(np.int64)
            ob = cb.offsets.cpu().numpy().astype(np.int64)
            da, db = ca.data.cpu().numpy(), cb.data.cpu().numpy()
            for i in np.nonzero(ok)[0][:4000]:
                assert bytes(da[oa[i]:oa[i + 1]]) == bytes(db[ob[i]:ob[i + 1]]), (ca.name, i)


@pytest.mark.parametrize('sizes', [[9000], [13, 1000, 7, 5003, 1], [8, 16, 4096], [3, 5, 11, 2000]])
def test_streamed_arrow_matches_whole_column_upload(sizes):
    import torch
    from spark_df_profiling import describe
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.ingest import from_arrow_streamed
    tab = _rechunk(_table(), sizes)
    dev = torch.device('cuda')
    whole = DeviceTable.from_arrow(tab.combine_chunks(), dev, streamed=False)
    stats = {}
    streamed = from_arrow_streamed(tab, dev, stats=stats)
    assert stats['rows'] == tab.num_rows and stats['h2d_bytes'] > 0
    _assert_same_buffers(whole, streamed)
    import oracle
    assert_describe_equal(describe(streamed, plots=False), oracle.describe(tab.combine_chunks()))


def test_parquet_round_trip(tmp_path):
    import torch
    from spark_df_profiling import describe
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.ingest import from_parquet
    tab = _table(12_345, seed=3)
    path = tmp_path / 't.parquet'
    pq.write_table(tab, path, row_group_size=3000)
    dev = torch.device('cuda')
    got = from_parquet(str(path), device=dev, batch_rows=1000)
    want = DeviceTable.from_arrow(pq.read_table(path), dev, streamed=False)
    _assert_same_buffers(want, got)
    import oracle
    assert_describe_equal(describe(str(path), plots=False), oracle.describe(pq.read_table(path)))
    sub = from_parquet(str(path), columns=['word', 'f64'], device=dev)
    assert sub.column_names == ['word', 'f64']


def test_profile_report_to_file(tmp_path):
    """ProfileReport(df).to_file() end to end on the GPU path (__init__.py:19-124)."""
    import datagen
    from spark_df_profiling import ProfileReport
    t = datagen.demo_like_table(20_000)
    rep = ProfileReport(t, sample=5)
    out = tmp_path / 'r.html'
    rep.to_file(str(out))
    text = out.read_text(encoding='utf8')
    assert text.startswith('<!doctype html>') and 'Dataset info' in text
    assert 'data:image/png;base64' in text                  # histograms rendered
    assert set(rep.get_description()) == {'table', 'variables', 'freq'}
    assert 'reclat_city' in rep.get_rejected_variables(0.9)


def _ragged_batches(tab, sizes):
    """tab's rows as a generator of RecordBatches of cycling (odd) sizes."""
    start = 0
    while start < tab.num_rows:
        for m in sizes:
            if start >= tab.num_rows:
                return
            for b in tab.slice(start, m).to_batches():
                yield b
            start += m


class _SparkStream:
    """A Spark DataFrame duck type whose Arrow transfer is an ITERATOR of
    RecordBatches of ragged sizes (Spark 3.x _collect_as_arrow batches as they
    arrive), with df.count() and df.dtypes (describe.py:71,137)."""

    def __init__(self, tab, sizes, dtypes=None):
        self._t, self._sizes = tab, sizes
        self.dtypes = dtypes if dtypes is not None else [
            (f.name, __import__('spark_df_profiling.columns', fromlist=['x']).spark_type_string(f.type))
            for f in tab.schema]
        self.pulled = 0

    def count(self):
        return self._t.num_rows

    def _collect_as_arrow(self):
        for b in _ragged_batches(self._t, self._sizes):
            self.pulled += 1
            yield b

    def limit(self, n):
        return _SparkStream(self._t.slice(0, n), self._sizes, self.dtypes)

    def toPandas(self):
        return self._t.to_pandas()


_SparkStream.__module__ = 'pyspark.sql.dataframe'


@pytest.mark.parametrize('sizes', [[70_001, 3, 12_345, 8], [1000, 9, 4096, 17]])
def test_streamed_spark_batches_vs_oracle(sizes):
    """§8(f3): a Spark-like DataFrame's batch iterator goes straight into the
    pinned double-buffered stager (no host concatenation; device buffers grow
    from 64 K rows when the stream's length is unknown), ragged batch sizes,
    every column type -- describe() equals the oracle on the same rows."""
    import oracle
    from spark_df_profiling import ProfileReport, describe
    tab = _table(150_003, seed=11)
    want = oracle.describe(tab)
    sdf = _SparkStream(tab, sizes)
    assert_describe_equal(describe(sdf, plots=False), want)
    assert sdf.pulled > 3                                       # consumed batch by batch
    # a bare iterator of batches (no count: buffers grow) and a RecordBatchReader
    assert_describe_equal(describe(_ragged_batches(tab, sizes), plots=False), want)
    reader = pa.RecordBatchReader.from_batches(tab.schema, _ragged_batches(tab, sizes))
    assert_describe_equal(describe(reader, plots=False), want)
    rep = ProfileReport(_ragged_batches(tab, sizes), sample=7)
    assert_describe_equal(rep.get_description(), oracle.describe(tab))
    assert 'Dataset info' in rep.to_html()


def test_spark_dtypes_dispatch():
    """describe.py:137 dispatches on Spark's df.dtypes strings: a column Spark
    types as decimal(12,2) is never 'decimal', so it is profiled as CAT/UNIQUE
    (describe.py:158-164) -- whatever the Arrow transfer looked like."""
    from spark_df_profiling import describe
    tab = _table(20_000, seed=5).select(['f64', 'dec', 'word'])
    sdf = _SparkStream(tab, [4096, 77], dtypes=[('f64', 'double'), ('dec', 'decimal(12,2)'), ('word', 'string')])
    d = describe(sdf, plots=False)
    assert d['variables'].loc['dec', 'type'] in ('CAT', 'UNIQUE')
    bad = _SparkStream(tab, [4096], dtypes=[('f64', 'double'), ('dec', 'decimal(12,2)'), ('word', 'bigint')])
    with pytest.raises(TypeError, match='word'):
        describe(bad, plots=False)
