"""Edge paths of the GPU engine that the ordinary tables never reach:

* the quantile window-miss and candidate-slot-overflow fallbacks (the
  missed rank's key range re-collected by sdp_column_keys_range, then an
  exact select), forced by the SDP_DEBUG_QUANTILE knob, against the oracle
  (test_gpu_scale_1e9.py repeats the forced miss at 1e9 rows);
* determinism: two describe() runs of one table are bitwise
  equal in every output;
* a duck-typed Spark DataFrame (toArrow / limit().toPandas()) through
  describe() and ProfileReport (reference __init__.py:61-68).
Needs an MI355X.
"""

import math

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

import datagen
from compare import assert_describe_equal

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('mode', ['overflow', 'miss'])
def test_quantile_fallback(monkeypatch, mode):
    import oracle
    from spark_df_profiling import describe, engine
    monkeypatch.setattr(engine, 'DEBUG_QUANTILE', mode)
    t = datagen.numeric_table(200_003, seed=17)
    raw = {}
    got = describe(t, raw=raw, plots=False)
    want = oracle.describe(t)
    assert_describe_equal(got, want)
    used = [name for name, b in raw['columns'].items() if 'numeric' in b and b['numeric'].fallback_used]
    assert used, 'the knob must route quantiles through the fallback'


def _bitwise_equal(a, b):
    if isinstance(a, pd.Series) or isinstance(b, pd.Series):
        return (isinstance(a, pd.Series) and isinstance(b, pd.Series) and list(a.index) == list(b.index)
                and all(_bitwise_equal(x, y) for x, y in zip(a.tolist(), b.tolist())))
    if isinstance(a, (float, np.floating)) and isinstance(b, (float, np.floating)):
        return np.float64(a).tobytes() == np.float64(b).tobytes() or (math.isnan(a) and math.isnan(b))
    return type(a) == type(b) and a == b


def test_determinism_bitwise():
    from spark_df_profiling import describe
    for t in (datagen.numeric_table(300_007, seed=23), datagen.categorical_table(120_000, seed=29),
              datagen.corr_table(100_000, seed=31)):
        r1, r2 = {}, {}
        a = describe(t, plots=False, raw=r1)
        b = describe(t, plots=False, raw=r2)
        assert a['table'] == b['table'] or all(_bitwise_equal(a['table'][k], b['table'][k]) for k in a['table'])
        va, vb = a['variables'], b['variables']
        assert list(va.index) == list(vb.index) and list(va.columns) == list(vb.columns)
        for name in va.index:
            for k in va.columns:
                assert _bitwise_equal(va.loc[name, k], vb.loc[name, k]), (name, k, va.loc[name, k], vb.loc[name, k])
        for k in a['freq']:
            assert _bitwise_equal(a['freq'][k], b['freq'][k]), k
        if r1['corr'] is not None:
            assert r1['corr'].to_numpy().tobytes() == r2['corr'].to_numpy().tobytes()


class _FakeSparkFrame:
    """The part of pyspark.sql.DataFrame the boundary touches: toArrow()
    (Spark >= 4; _collect_as_arrow() on 3.x) and limit(n).toPandas()."""

    def __init__(self, table):
        self._t = table

    def toArrow(self):
        return self._t

    def limit(self, n):
        return _FakeSparkFrame(self._t.slice(0, n))

    def toPandas(self):
        return self._t.to_pandas()


_FakeSparkFrame.__module__ = 'pyspark.sql.dataframe'


class _FakeSparkFrame3(_FakeSparkFrame):
    toArrow = None

    def _collect_as_arrow(self):
        return self._t.to_batches(max_chunksize=4096)


_FakeSparkFrame3.__module__ = 'pyspark.sql.dataframe'


def test_spark_like_input(tmp_path):
    import oracle
    from spark_df_profiling import ProfileReport, describe
    t = datagen.demo_like_table(20_000)
    want = oracle.describe(t)
    assert_describe_equal(describe(_FakeSparkFrame(t), plots=False), want)
    assert_describe_equal(describe(_FakeSparkFrame3(t), plots=False), want)
    rep = ProfileReport(_FakeSparkFrame(t))
    out = tmp_path / 'spark_like.html'
    rep.to_file(str(out))
    html = out.read_text(encoding='utf8')
    assert 'data:image/png' in html and 'reclat_city' in html
    with pytest.raises(TypeError):
        describe(object())


def test_int32_extremes_at_window_bounds():
    """4-byte integer columns whose quantile windows start at the type's
    smallest key (INT32_MIN, 0u) or end at its largest (INT32_MAX,
    UINT32_MAX), with nulls: pass 1's 32-bit window test must not take the
    null rows' key 0 as candidates, nor drop the maximum (sdp_numeric.hip,
    pass1_body's lo32/hi32; describe.py:203-208 percentiles)."""
    import oracle
    from spark_df_profiling import describe
    rng = np.random.default_rng(41)
    for n in (97, 300, 5000):
        a = rng.integers(-100, 100, n).astype(np.int32)
        a[rng.integers(0, n)] = np.iinfo(np.int32).min
        a[rng.integers(0, n)] = np.iinfo(np.int32).max
        u = rng.integers(0, 100, n).astype(np.uint32)
        u[rng.integers(0, n)] = 0
        u[rng.integers(0, n)] = np.iinfo(np.uint32).max
        lo_only = rng.integers(-100, 100, n).astype(np.int32)
        lo_only[rng.permutation(n)[:3]] = np.iinfo(np.int32).min + np.arange(3)
        masks = [rng.random(n) < 0.15 for _ in range(3)]
        t = pa.table({'i32': pa.array(a, mask=masks[0]), 'u32': pa.array(u, mask=masks[1]),
                      'i32_low': pa.array(lo_only, mask=masks[2])})
        assert_describe_equal(describe(t, plots=False), oracle.describe(t))


def test_uint32_wide_fused_group(monkeypatch):
    """Eight or more high-cardinality uint32 columns (dtype SDP_U32, range over
    2^20, 64 K..2^26 rows) take the fused wide-table distinct-count path
    (engine._group_middle_fused -> sdp_part_rows_batch), describe.py:143."""
    import oracle
    from spark_df_profiling import describe
    rng = np.random.default_rng(43)
    n = 100_000
    cols = {}
    for j in range(9):
        v = rng.integers(0, 2 ** 32, n, dtype=np.uint64).astype(np.uint32)
        v[:n // 40] = v[n // 2:n // 2 + n // 40]          # repeats: distinct < rows, still near-unique
        cols['u%d' % j] = pa.array(v, mask=rng.random(n) < 0.05)
    t = pa.table(cols)
    from spark_df_profiling import engine as engmod
    from spark_df_profiling.engine import Engine
    monkeypatch.setattr(engmod, 'BITS32', False)        # (uint32 keys would take sdp_distinct32)
    fused = []
    orig = Engine._group_middle_fused

    def spy(self, ctxs, bsns):
        fused.append([c['col'].dtype for c in ctxs])
        return orig(self, ctxs, bsns)
    monkeypatch.setattr(Engine, '_group_middle_fused', spy)
    assert_describe_equal(describe(t, plots=False), oracle.describe(t))
    assert fused and all(d == 9 for grp in fused for d in grp), fused     # SDP_U32 = 9
