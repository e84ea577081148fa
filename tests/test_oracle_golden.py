"""The CPU oracle against the reference's own known answers (CPU only)."""

import json
import math
import os

import numpy as np
import pytest

import datagen
import oracle

HERE = os.path.dirname(os.path.abspath(__file__))
KNOWN = json.load(open(os.path.join(HERE, 'golden', 'known_answers.json')))


@pytest.fixture(scope='module')
def legacy():
    return oracle.profile_raw(datagen.legacy_table())


def _eq(a, b):
    if isinstance(b, float):
        return math.isclose(float(a), b, rel_tol=1e-13, abs_tol=1e-15)
    return a == b


@pytest.mark.parametrize('col', ['x', 'y', 'cat', 's1', 's2', 'id', 'somedate'])
def test_column_known_answers(legacy, col):
    d, raw = legacy
    row = d['variables'].loc[col]
    for k, v in KNOWN[col].items():
        if k == 'hist_edges':
            assert raw['columns'][col]['hist']['edges'] == v
        elif k == 'hist_counts':
            assert list(raw['columns'][col]['hist']['counts']) == v
        else:
            assert _eq(row[k], v), (col, k, row[k], v)


def test_table_known_answers(legacy):
    d, _ = legacy
    for k, v in KNOWN['table'].items():
        assert _eq(d['table'][k], v), (k, d['table'][k], v)


def test_keys_and_freq(legacy):
    d, _ = legacy
    assert set(d) == {'table', 'variables', 'freq'}
    assert set(d['freq']) == {'id', 'cat', 's1', 's2'}        # CAT / UNIQUE / CONST only
    vc = d['freq']['cat']
    assert list(vc.index[-2:]) == ['***Other Values***', '***Other Values Distinct Count***']
    assert vc.iloc[0] == 3 and vc.index[0] == 'c'


def test_pandas_typed_x_is_double():
    """As pandas->Spark would type it, x is double with NaN: distinct counts the
    NaN (7, the legacy expectation) and quantiles are data elements."""
    d = oracle.describe(datagen.legacy_table_pandas_typed())
    v = d['variables'].loc['x']
    assert v['distinct_count'] == 7 and v['count'] == 8
    assert v['p_unique'] == 7 / 8
    assert [v[k] for k in ('5%', '25%', '50%', '75%', '95%')] == [-10.0, -3.0, 0.0, 15.0, 50.0]


def test_no_numeric_column_raises_keyerror():
    """describe.py:108 reads variable_stats.ix['high_idx'] (App. C quirk)."""
    import pyarrow as pa
    with pytest.raises(KeyError):
        oracle.describe(pa.table({'s': pa.array(['a', 'b', 'b'])}))


def test_bins_one_raises():
    with pytest.raises(IndexError):
        oracle.describe(datagen.legacy_table(), bins=1)


def test_corr_reject_order():
    d = oracle.describe(datagen.corr_table(3000))
    v = d['variables']
    assert v.loc['b', 'type'] == 'CORR' and v.loc['b', 'correlation_var'] == 'a'
    assert v.loc['e', 'type'] == 'CORR'
    assert d['table']['REJECTED'] == d['table']['CONST'] + d['table']['CORR']


def _accumulate(lo, hi, bins=10):
    w = (hi - lo) / float(bins)
    e, out = lo, []
    for _ in range(bins):
        out.append(e)
        e = e + w
    return out


def test_range_and_edges_are_float64_after_the_row_upcast():
    """describe.py:209 `stats_df.ix[0]` turns the mixed int64 / float32 /
    float64 agg row into one float64 Series before :211 (range) and :226
    (generate_hist_data), so min / max are float64 there.  SURVEY.md A.6's
    int64 (resp. float32) subtraction would give other ranges and edges on
    these columns; the oracle follows the upcast."""
    t = datagen.wide_range_table()
    d, raw = oracle.profile_raw(t)
    v = d['variables']
    # int64 beyond 2^53: float64(max) - float64(min) != float(int(max) - int(min))
    import pyarrow.compute as pc
    mm = pc.min_max(t.column('i64_big'))
    imax, imin = mm['max'].as_py(), mm['min'].as_py()
    assert abs(imax) > 2 ** 53 and abs(imin) > 2 ** 53
    assert v.loc['i64_big', 'range'] == float(imax) - float(imin)
    assert float(imax) - float(imin) != float(imax - imin)
    assert raw['columns']['i64_big']['hist']['edges'] == _accumulate(float(imin), float(imax))
    assert _accumulate(float(imin), float(imax)) != [float(e) for e in _accumulate(imin, imax)]
    # float32: the range in float32 rounds differently
    mm = pc.min_max(t.column('f32_range'))
    fmax, fmin = np.float32(mm['max'].as_py()), np.float32(mm['min'].as_py())
    assert v.loc['f32_range', 'range'] == float(fmax) - float(fmin)
    assert float(np.float32(fmax - fmin)) != float(fmax) - float(fmin)
    assert raw['columns']['f32_range']['hist']['edges'] == _accumulate(float(fmin), float(fmax))
    # the int64 sum wraps (Spark LongType Sum) and is compared exactly
    w = t.column('i64_wrap')
    wv = np.asarray(pc.drop_null(w).to_numpy(), dtype=np.int64)
    s = int(np.sum(wv, dtype=np.int64))
    assert abs(sum(int(x) for x in wv)) >= 2 ** 63          # it did wrap
    assert v.loc['i64_wrap', 'sum'] == float(s)
    assert set(v.attrs['integral_num']) >= {'i64_big', 'i64_wrap'}
