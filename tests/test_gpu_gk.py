"""Spark 2.x percentile_approx emulation on the GPU (sdp_gk_quantiles,
describe(quantile_mode='gk')) against the CPU restatement oracle/gk.py, bit
for bit: multi-batch partitions (50000-value heads), several partitions,
nulls, NaN, +-0.0, heavy duplicates, f32 and f64, low accuracy.  Parity with
Spark itself is unpinned (no Spark here); both sides are checked against
Spark's documented rank window in tests/test_gk_oracle.py.  Needs an MI355X."""

import math
import zlib

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

PROBS = [0.05, 0.25, 0.5, 0.75, 0.95]


def _column(values, valid):
    from spark_df_profiling.columns import DeviceTable
    arr = pa.array(values, mask=None if valid is None else ~valid)
    return DeviceTable.from_arrow(pa.table({'x': arr})).columns[0]


def _same(a, b):
    return (math.isnan(a) and math.isnan(b)) or (a == b and math.copysign(1, a) == math.copysign(1, b))


@pytest.mark.parametrize('case', ['f64_norm_3p', 'f64_nulls_nan_zeros_1p', 'f32_dups_4p', 'f64_acc100_2p',
                                  'f64_lognormal_many_heads_2p'])
def test_gk_matches_restatement(case):
    from oracle import gk
    from spark_df_profiling.engine import Engine
    rng = np.random.default_rng(zlib.crc32(case.encode()))
    acc, parts, valid = 10000, 1, None
    if case == 'f64_norm_3p':
        vals, parts = rng.standard_normal(160_003), 3
    elif case == 'f64_nulls_nan_zeros_1p':
        vals = rng.standard_normal(120_001)
        vals[rng.random(vals.size) < 0.05] = np.nan
        z = rng.random(vals.size) < 0.02
        vals[z] = np.where(rng.random(z.sum()) < 0.5, -0.0, 0.0)
        valid = rng.random(vals.size) >= 0.05
    elif case == 'f32_dups_4p':
        vals, parts = rng.integers(-20, 20, 110_000).astype(np.float32), 4
    elif case == 'f64_acc100_2p':
        vals, parts, acc = rng.exponential(1.0, 101_000), 2, 100
    else:                    # five full 50000-value heads per partition: insert + compress rounds
        vals, parts = rng.lognormal(0.0, 2.0, 520_000), 2
    col = _column(vals, valid)
    got = Engine().gk_quantiles(col, PROBS, partitions=parts, accuracy=acc)
    want = gk.percentile_approx(gk.split_rows(vals, valid, parts), PROBS, accuracy=acc)
    for p, w in zip(PROBS, want):
        assert _same(got[p], float(w)), (case, p, got[p], w)


def test_describe_quantile_mode_gk():
    """describe(quantile_mode='gk'): float columns take the emulated elements
    (and their q1/q3 for high_idx/low_idx, describe.py:212-223); integral
    columns keep the exact percentile."""
    from oracle import gk
    from spark_df_profiling import describe
    rng = np.random.default_rng(11)
    n = 100_003
    x = rng.standard_normal(n)
    k = rng.integers(0, 1000, n)
    t = pa.table({'x': x, 'k': k})
    got = describe(t, plots=False, quantile_mode='gk', spark_partitions=2)
    want = gk.percentile_approx(gk.split_rows(x, None, 2), PROBS)
    v = got['variables']
    for p, w in zip(PROBS, want):
        key = '%d%%' % int(p * 100)
        assert v.loc['x', key] == w
    q1, q3 = want[1], want[3]
    assert v.loc['x', 'high_idx'] == int((x > q3 + 2 * (q3 - q1)).sum())
    assert v.loc['x', 'low_idx'] == int((x < q1 - 2 * (q3 - q1)).sum())
    exact = describe(t, plots=False)['variables']
    for p in PROBS:
        key = '%d%%' % int(p * 100)
        assert v.loc['k', key] == exact.loc['k', key]
