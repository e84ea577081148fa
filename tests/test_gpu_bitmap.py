"""Small-range countDistinct through the LDS-bitmap kernels (sdp_bitmap.hip)
vs numpy, exact: every integral width, nulls, sliced (bit-offset) validity,
ragged lengths, and ranges at the 2^20 limit.  Needs an MI355X."""

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu


def _distinct_gpu(arr):
    import torch
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.engine import Engine
    t = DeviceTable.from_arrow(pa.table({'c': arr}), torch.device('cuda'))
    col = t.columns[0]
    e = Engine()
    p1 = e.minmax_pass(col)
    lo, rng = p1['imin'], p1['imax'] - p1['imin'] + 1
    return e.distinct_bitmap(col, lo, rng), rng


def _want(arr):
    v = arr.drop_null().to_numpy(zero_copy_only=False)
    return len(np.unique(v))


@pytest.mark.parametrize('typ,lo,hi', [(pa.int8(), -128, 128), (pa.int16(), -3000, 3000), (pa.int32(), -5, 70_000),
                                       (pa.int64(), 10 ** 12, 10 ** 12 + 500_000), (pa.uint8(), 0, 256),
                                       (pa.uint16(), 0, 65536), (pa.uint32(), 4_000_000_000, 4_000_900_000),
                                       (pa.date32(), -100_000, 50_000)])
@pytest.mark.parametrize('n', [1, 17, 100_003, 3_000_001])
def test_bitmap_distinct(typ, lo, hi, n):
    g = np.random.default_rng(n + hi % 1000)
    vals = g.integers(lo, hi, n)
    mask = g.random(n) < 0.07
    if pa.types.is_date32(typ):
        arr = pa.array(vals.astype(np.int32), type=pa.int32(), mask=mask).cast(pa.date32())
    else:
        arr = pa.array(vals, mask=mask).cast(typ)
    if arr.null_count == len(arr):
        return
    got, rng = _distinct_gpu(arr)
    assert rng <= 1 << 20
    assert got == _want(arr)


@pytest.mark.parametrize('span', [(1 << 20) - 1, 1 << 20])
def test_bitmap_range_limit(span):
    g = np.random.default_rng(3)
    v = g.integers(0, span, 2_000_000)
    v[0], v[1] = 0, span - 1                 # pin the range exactly
    arr = pa.array(v - 777)
    got, rng = _distinct_gpu(arr)
    assert rng == span
    assert got == len(np.unique(v))


def test_bitmap_sliced_validity():
    g = np.random.default_rng(9)
    v = g.integers(-50_000, 50_000, 1_000_003)
    arr = pa.array(v, mask=g.random(len(v)) < 0.2).slice(13, 900_001)
    got, _ = _distinct_gpu(arr)
    assert got == _want(arr)
