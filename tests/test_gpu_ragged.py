"""describe() on ragged, sliced and multi-chunk Arrow tables vs the CPU oracle.

Row counts around the kernels' vector and tile boundaries exercise the tail
paths (pass 1's n % VPT tail, partially filled tiles, one-element windows);
sliced tables carry non-zero Arrow offsets into the validity bitmaps and value
buffers; concatenated tables arrive as several chunks per column.  A one-row
table has no NUM column, so the reference's describe() raises KeyError at
describe.py:108 -- the HIP path must raise the same.  Needs an MI355X.
"""

import pyarrow as pa
import pytest

import datagen
from compare import assert_describe_equal
from test_gpu_parity import _check_hist, _run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('n', [2, 3, 5, 17, 63, 65, 257, 1025, 4099])
def test_ragged_row_counts(n):
    got, raw, want, want_raw = _run(datagen.numeric_table(n, seed=n))
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_sliced_numeric():
    got, raw, want, want_raw = _run(datagen.numeric_table(5000).slice(37, 3001))
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_sliced_categorical():
    got, raw, want, want_raw = _run(datagen.categorical_table(4000).slice(13, 2501))
    assert_describe_equal(got, want)


def test_multi_chunk():
    t = pa.concat_tables([datagen.numeric_table(1000, seed=1), datagen.numeric_table(777, seed=2)])
    assert t.column(0).num_chunks == 2
    got, raw, want, want_raw = _run(t)
    assert_describe_equal(got, want)
    _check_hist(raw, want_raw)


def test_one_row_raises_like_reference():
    import oracle
    from spark_df_profiling import describe
    t = datagen.numeric_table(1, seed=1)
    with pytest.raises(KeyError):
        oracle.profile_raw(t)
    with pytest.raises(KeyError):
        describe(t, plots=False)
