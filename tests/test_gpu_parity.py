"""describe() on the HIP path vs the CPU oracle, on the same seeded Arrow tables.

Every statistic of the reference's output dict is compared (tests/compare.py
states the tolerances); exact histogram bin counts are compared through the
`raw` side channel.  Needs an MI355X.
"""

import numpy as np
import pytest

import datagen
from compare import assert_describe_equal

pytestmark = pytest.mark.gpu


def _run(table, **kw):
    import oracle
    from spark_df_profiling import describe
    raw = {}
    got = describe(table, raw=raw, plots=False, **kw)
    want, want_raw = oracle.profile_raw(table, **kw)
    return got, raw, want, want_raw


def _check_hist(raw, want_raw):
    for name, w in want_raw['columns'].items():
        if 'hist' not in w:
            continue
        st = raw['columns'][name]['numeric']
        assert np.array_equal(np.asarray(st.hist_counts), w['hist']['counts']), name
        assert [float(e) for e in st.edges] == [float(e) for e in w['hist']['edges']], name


@pytest.mark.parametrize('maker', [datagen.legacy_table, datagen.legacy_table_pandas_typed,
                                   datagen.small_edge_table, datagen.wide_range_table])
def test_small_tables(maker):
    got, raw, want, want_raw = _run(maker())
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_legacy_known_answers():
    """Spark-valid values recomputed from tests.py.old.py:58-76."""
    from spark_df_profiling import describe
    d = describe(datagen.legacy_table(), plots=False)
    v = d['variables']
    assert v.loc['x', 'mean'] == 13.375
    assert v.loc['x', 'variance'] == 561.125
    assert abs(v.loc['x', 'skewness'] - 0.8700654233008702) < 1e-15
    assert abs(v.loc['x', 'kurtosis'] - (-0.9061564710904944)) < 1e-15
    assert [v.loc['x', k] for k in ('5%', '25%', '50%', '75%', '95%')] == [-7.549999999999999, -0.75, 2.5, 23.75, 50.0]
    assert v.loc['x', 'mad'] == 18.71875
    assert v.loc['x', 'distinct_count'] == 6 and v.loc['x', 'count'] == 8
    assert abs(v.loc['y', 'skewness'] - 2.097192909339155) < 1e-14
    assert abs(v.loc['y', 'kurtosis'] - 2.654350961293982) < 1e-14
    assert d['table']['total_missing'] == pytest.approx(0.063492063492063489, abs=1e-15)


@pytest.mark.parametrize('n', [1000, 200_003])
def test_numeric_mix(n):
    got, raw, want, want_raw = _run(datagen.numeric_table(n))
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_categorical():
    got, raw, want, want_raw = _run(datagen.categorical_table(50_000))
    assert_describe_equal(got, want)


def test_dates():
    got, raw, want, want_raw = _run(datagen.date_table(20_000))
    assert_describe_equal(got, want)


def test_corr_reject():
    got, raw, want, want_raw = _run(datagen.corr_table(30_000))
    assert_describe_equal(got, want)
    assert got['table']['CORR'] == want['table']['CORR'] > 0
    g = raw['corr'].to_numpy()
    w = want_raw['corr'].to_numpy()
    assert np.allclose(g, w, rtol=1e-9, atol=1e-12)


def test_demo_like_config1():
    got, raw, want, want_raw = _run(datagen.demo_like_table(100_000))
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_bins_100_and_k_vals():
    t = datagen.numeric_table(20_000, seed=3)
    got, raw, want, want_raw = _run(t, bins=100, k_vals={'f64_norm': 1.5, 'i64_small': 0})
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_errors():
    import pyarrow as pa
    from spark_df_profiling import describe
    with pytest.raises(TypeError):
        describe([1, 2, 3])
    with pytest.raises(ValueError):
        describe(pa.table({'a': pa.array([], pa.int64())}))
    with pytest.raises(NotImplementedError):
        describe(pa.table({'a': pa.array([[1], [2]])}))
    with pytest.raises(IndexError):
        describe(datagen.legacy_table(), bins=1)
