"""sdp_pass2_gram -- pass 2 of every NUM column and the Pearson Gram in one
read (describe.py:215-223, :49; utils.py:27-31) -- against the oracle and
against the separate launches (sdp_pass2_count_batch + sdp_rowmask +
sdp_gram) it replaces: mixed f64 / f32 / i64 / i32 columns with nulls, NaN,
+-0.0, a constant and an all-null column (outside the Pearson set), partition
counts with heavy keys, 32-bit key spaces and columns without a level-1 count,
row counts around the 16-row k-blocks and the partition row blocks.  Needs an
MI355X."""

import numpy as np
import pyarrow as pa
import pytest

import datagen
from compare import assert_describe_equal, close

pytestmark = pytest.mark.gpu


def _table(n, seed, heavy_cols=1):
    g = datagen.rng(seed)
    cols = {}

    def nulls(p=0.05):
        return g.random(n) < p
    f = g.standard_normal(n)
    f[g.random(n) < 0.01] = np.nan
    f[g.random(n) < 0.01] = -0.0
    cols['f64_nan'] = pa.array(f, mask=nulls())
    cols['f64_shift'] = pa.array(1e9 + g.standard_normal(n), mask=nulls())
    cols['f32_u'] = pa.array(g.random(n).astype(np.float32), mask=nulls())
    cols['i64_wide'] = pa.array(g.integers(-2 ** 40, 2 ** 40, n), mask=nulls())
    cols['i64_small'] = pa.array(g.integers(0, 1000, n), mask=nulls())          # LDS bitmap: no count in pass 2
    cols['i32_range'] = pa.array(g.integers(-2 ** 31, 2 ** 31 - 1, n).astype(np.int32), mask=nulls())
    for h in range(heavy_cols):                                                  # skewed: heavy keys
        cols['i64_zipf%d' % h] = pa.array(np.minimum(g.zipf(1.2 + 0.1 * h, n), 10 ** 9).astype(np.int64),
                                          mask=nulls())
    cols['const'] = pa.array(np.full(n, 7.5))                                   # CONST: outside the Pearson set
    cols['all_null'] = pa.array(np.zeros(n), mask=np.ones(n, dtype=bool))
    cols['f64_corr'] = pa.array(np.nan_to_num(f, nan=0.0) * 0.5 + g.standard_normal(n) * 0.1, mask=nulls(0.02))
    return pa.table(cols)


def _run(table, fused, monkeypatch):
    from spark_df_profiling import _native as nat
    from spark_df_profiling import describe
    from spark_df_profiling.engine import Engine
    monkeypatch.setattr(Engine, 'P2GRAM', fused)
    rec = nat.start_recording()
    try:
        got = describe(table, plots=False, raw=(raw := {}))
    finally:
        nat.stop_recording()
    return got, raw, {k.split('[')[0] for k in rec}


# (heavy=1: f64_nan's NaN / 0.0 keys are heavy too, so both LDS heavy tables are used)
@pytest.mark.parametrize('n,heavy', [(300_007, 1), (70_001, 0), (4_099, 0)])
def test_pass2_gram_matches_oracle_and_separate_path(n, heavy, monkeypatch):
    import oracle
    t = _table(n, 90 + n % 97 + heavy, heavy)
    got, raw, called = _run(t, True, monkeypatch)
    assert 'sdp_pass2_gram' in called and 'sdp_gram' not in called, called
    want, wraw = oracle.profile_raw(t)
    assert_describe_equal(got, want)
    sep, sraw, called2 = _run(t, False, monkeypatch)
    assert 'sdp_pass2_gram' not in called2 and 'sdp_gram' in called2
    # integer outputs bit-identical to the separate launches; the Pearson
    # matrix equal up to the Gram's summation order
    for name, a in raw['columns'].items():
        st, ss = a.get('numeric'), sraw['columns'][name].get('numeric')
        if st is None:
            continue
        assert (st.high_idx, st.low_idx) == (ss.high_idx, ss.low_idx), name
        assert list(map(int, st.hist_counts)) == list(map(int, ss.hist_counts)), name
        assert close(st.mad, ss.mad, rel=1e-13), name
    assert got['variables']['distinct_count'].to_dict() == sep['variables']['distinct_count'].to_dict()
    ca, cb = raw['corr'], sraw['corr']
    assert list(ca.index) == list(cb.index) and 'const' not in ca.index and 'all_null' not in ca.index
    assert np.allclose(ca.to_numpy(), cb.to_numpy(), rtol=1e-12, atol=1e-14, equal_nan=True)
    wc = wraw['corr'].loc[ca.index, ca.columns].to_numpy()
    for x, y in zip(ca.to_numpy().ravel(), wc.ravel()):
        assert close(x, y) or (np.isnan(x) and np.isnan(y))


def test_pass2_gram_falls_back_beyond_two_heavy_columns(monkeypatch):
    """Three skewed columns (plus f64_nan's heavy NaN / 0.0 keys): more heavy
    tables than the kernel holds -> the separate launches, same results."""
    import oracle
    t = _table(200_003, 7, heavy_cols=3)
    got, raw, called = _run(t, True, monkeypatch)
    assert 'sdp_pass2_gram' not in called and 'sdp_gram' in called
    want, _ = oracle.profile_raw(t)
    assert_describe_equal(got, want)


def test_pass2_gram_no_corr(monkeypatch):
    """corr_reject=None: no Pearson matrix is asked for, pass 2 stays separate."""
    from spark_df_profiling import _native as nat
    from spark_df_profiling import describe
    import oracle
    t = _table(100_003, 8, 0)
    rec = nat.start_recording()
    try:
        got = describe(t, plots=False, corr_reject=None)
    finally:
        nat.stop_recording()
    assert not any(k.startswith('sdp_pass2_gram') or k.startswith('sdp_gram') for k in rec)
    want = oracle.describe(t, corr_reject=None)
    assert_describe_equal(got, want)
