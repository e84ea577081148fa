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
