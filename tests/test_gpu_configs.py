"""describe() on the BASELINE.json configurations vs the oracle.

Each configuration's generator runs at the largest size the vectorised oracle
(oracle/fast.py, itself pinned to the exact restatement by
test_oracle_fast.py) checks within a test's time budget:

  C1  Demo-like mixed 10 columns            1e6 rows
  C3  the bench table (16 mixed, 5 % nulls)  4 M rows (bench.make_c3_shard)
  C4  near-unique int64 + zipf hex ids       4 M rows (exact distinct, top-50)
  C5  512 fp32 columns, Pearson on MFMA      2e5 rows (+ numpy fp64 Gram)

Every statistic is compared (tests/compare.py tolerances), histogram bins
exactly.  C2 runs at its full 1e8 rows, and C4/C5 at their full sizes, in
test_gpu_baseline_sizes.py.  Needs an MI355X.
"""

import numpy as np
import pytest

import datagen
from compare import assert_describe_equal

pytestmark = pytest.mark.gpu


def _check(table_for_gpu, table_arrow, **kw):
    import torch
    from oracle import fast
    from spark_df_profiling import describe
    raw = {}
    got = describe(table_for_gpu, raw=raw, plots=False, **kw)
    torch.cuda.synchronize()
    want, want_raw = fast.profile_raw(table_arrow, **kw)
    assert_describe_equal(got, want)
    for name, w in want_raw['columns'].items():
        if 'hist' in w:
            st = raw['columns'][name]['numeric']
            assert np.array_equal(np.asarray(st.hist_counts), w['hist']['counts']), name
    return got, raw, want, want_raw


def test_c1_demo_like_1e6():
    t = datagen.demo_like_table(1_000_000)
    got, raw, want, want_raw = _check(t, t)
    assert got['table']['CONST'] == 1 and got['table']['DATE'] == 1


def test_c3_bench_table_4m():
    import torch
    import bench
    dev = torch.device('cuda', 0)
    shard = bench.make_c3_shard(4_000_000, 0, 1, dev)
    t = bench.shard_to_arrow(shard)
    _check(shard, t)


def test_c4_high_cardinality_4m():
    t = datagen.c4_table(4_000_000)
    got, raw, want, want_raw = _check(t, t)
    assert got['variables'].loc['hex_id', 'type'] == 'CAT'
    assert len(got['freq']['hex_id']) == 52                 # top-50 + the two "Other" rows


def test_c5_wide_pearson_2e5():
    import torch
    t = datagen.c5_table(200_000)
    torch.cuda.reset_peak_memory_stats()
    got, raw, want, want_raw = _check(t, t)
    g = raw['corr'].to_numpy()
    w = want_raw['corr'].to_numpy()
    assert g.shape == (512, 512)
    assert np.allclose(g, w, rtol=1e-9, atol=1e-12)
    # wide tables keep candidate-slot memory bounded (engine.CAND_FULL_BUDGET:
    # 1 GiB of room-for-every-row slots per pass-1 batch, sample-sized beyond)
    table_bytes = 200_000 * 512 * 4
    assert torch.cuda.max_memory_allocated() < 3 * table_bytes + (7 << 29)
