"""countDistinct of sorted columns (describe.py:143) through the one-pass
sdp_sorted_distinct path, against the oracle: columns the pass-1 sample finds
non-decreasing are verified in one streaming read; a decrease the sample
missed, or a null run longer than the kernel's walk, falls back to the
partitioning path -- either way the counts must equal the oracle's.
Needs an MI355X."""

import pytest

import datagen
from compare import assert_describe_equal

pytestmark = pytest.mark.gpu


def test_sorted_columns_vs_oracle():
    from oracle import fast
    from spark_df_profiling import describe
    t = datagen.sorted_table(300_007)
    raw = {}
    # (the sorted columns correlate: corr_reject=None keeps their statistics)
    got = describe(t, raw=raw, plots=False, corr_reject=None)
    want, _ = fast.profile_raw(t, corr_reject=None)
    assert_describe_equal(got, want)
    sd = {name: b['p1'].get('sorted_distinct') for name, b in raw['columns'].items() if 'p1' in b}
    for name in ('ids', 'dup', 'fsort', 'f32sort'):
        assert sd[name] is not None, name                # taken by the sorted path
    for name in ('almost', 'nullrun', 'desc', 'num'):
        assert sd[name] is None, name                    # verified unsorted (or never a candidate): grouped


def _sorted_distinct(arr):
    import ctypes
    import pyarrow as pa
    import torch
    from spark_df_profiling import _native as nat
    from spark_df_profiling._native import sdp, ptr
    from spark_df_profiling.columns import DeviceTable
    t = DeviceTable.from_arrow(pa.table({'c': arr}))
    cs = t.columns[0].sdp()
    out = torch.zeros(4, dtype=torch.int64, device='cuda')
    sdp.sdp_sorted_distinct(ctypes.byref(cs), ptr(out), nat.stream_handle())
    return [int(x) & ((1 << 64) - 1) for x in out.cpu().tolist()]


@pytest.mark.parametrize('np_dtype', ['int8', 'int16', 'int32', 'int64', 'float32', 'float64'])
def test_sorted_distinct_kernel_lanes_and_null_runs(np_dtype):
    """sdp_sorted_distinct on crafted sorted columns: duplicates, null runs of
    1..200 rows placed across the 8-row lane groups and the 64-lane waves (the
    left-lane hand-off and the walk back), a ragged tail; then one decrease at
    a lane edge, one inside a lane, and a null run longer than the walk."""
    import numpy as np
    import pyarrow as pa
    g = datagen.rng(51)
    n = 200_003
    hi = {'int8': 120, 'int16': 30_000}.get(np_dtype, 60_000)
    v = np.sort(g.integers(-hi, hi, n)).astype(np_dtype)
    valid = np.ones(n, dtype=bool)
    for start, ln in ((0, 3), (7, 1), (63, 2), (511, 9), (1023, 64), (4096, 130), (9000, 200), (n - 5, 5)):
        valid[start:start + ln] = False
    for start in g.integers(0, n - 10, 300):
        valid[start:start + int(g.integers(1, 9))] = False

    def check(vals, ok, want_viol):
        d, viol, _, _ = _sorted_distinct(pa.array(vals, mask=~ok))
        assert viol == want_viol
        if not want_viol:
            assert d == len(np.unique(vals[ok]))
    check(v, valid, 0)
    w = v.copy()
    w[8 * 1000] = w[8 * 1000 - 1] - 1 if np_dtype != 'int8' else -hi - 1      # decrease at a lane edge
    valid2 = valid.copy()
    valid2[8 * 1000 - 1:8 * 1000 + 1] = True
    check(w, valid2, 1)
    w = v.copy()
    w[8 * 2000 + 3] = w[8 * 2000 + 2] - 1 if np_dtype != 'int8' else -hi - 1   # inside a lane
    valid3 = valid.copy()
    valid3[8 * 2000 + 2:8 * 2000 + 4] = True
    check(w, valid3, 1)
    valid4 = valid.copy()
    valid4[50_000:50_400] = False                                              # longer than the walk
    check(v, valid4, 1)
