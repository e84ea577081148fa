"""The vectorised oracle mode (oracle/fast.py) against the exact restatement.

The exact mode is pinned by the reference's known answers
(test_oracle_golden.py); this pins the vectorised mode -- used by the GPU
tests at the BASELINE configuration sizes and by bench.py's multi-core CPU
baseline -- to the exact one on every table family, including small versions
of the BASELINE configurations (C2, C4, C5)."""

import pytest

import datagen
import oracle
from compare import assert_describe_equal
from oracle import fast

TABLES = {
    'legacy': datagen.legacy_table,
    'legacy_pandas_typed': datagen.legacy_table_pandas_typed,
    'edge': datagen.small_edge_table,
    'numeric': lambda: datagen.numeric_table(30_011),
    'categorical': lambda: datagen.categorical_table(12_000),
    'dates': lambda: datagen.date_table(4_000),
    'corr': lambda: datagen.corr_table(6_000),
    'demo_c1': lambda: datagen.demo_like_table(15_000),
    'c2': lambda: datagen.c2_table(40_000),
    'c4': lambda: datagen.c4_table(40_000),
    'c5': lambda: datagen.c5_table(8_000, ncols=48),
}


@pytest.mark.parametrize('name', sorted(TABLES))
def test_fast_equals_exact(name):
    t = TABLES[name]()
    want, want_raw = oracle.profile_raw(t)
    got, got_raw = fast.profile_raw(t)
    assert_describe_equal(got, want)
    for col, w in want_raw['columns'].items():
        if 'hist' in w:
            assert list(got_raw['columns'][col]['hist']['counts']) == list(w['hist']['counts']), col


def test_fast_bins_and_k_vals():
    t = datagen.numeric_table(9_001, seed=3)
    kw = dict(bins=100, k_vals={'f64_norm': 1.5, 'i64_small': 0})
    assert_describe_equal(fast.describe(t, **kw), oracle.describe(t, **kw))


def test_config_generators_shapes():
    assert datagen.c2_table(1000).num_columns == 8
    t4 = datagen.c4_table(1000)
    assert t4.column('hex_id').type == __import__('pyarrow').string()
    assert all(len(x) == 16 for x in t4.column('hex_id').to_pylist()[:50])
    assert datagen.c5_table(100, ncols=512).num_columns == 512
