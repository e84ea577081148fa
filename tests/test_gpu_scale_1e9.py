"""The bench table itself (1e9 rows x 16 columns, bench.make_c3_shard) profiled
once, every NUM statistic re-derived by independent torch code on the same
device (tests/torch_ref.py: comparisons, sorts and exactly-added chunk sums,
no libsdp):

* count / n_missing from the validity bitmaps, min / max;
* mean, variance, std, skewness, kurtosis (two-pass fp64, Spark's population
  formulas), sum (int64 columns: wrapping Long sum), mad -- 1e-9 relative;
* histogram bins (#(x >= e_j) differences on the host-accumulated edges),
  n_zeros, high/low outlier counts -- exact;
* float quantiles: the element of rank ceil(pN); int quantiles: Spark's
  Percentile interpolation on the exact order statistics (torch.unique) --
  exact; int distinct counts (torch.unique) -- exact;
* distinct counts of f32_uniform and date (torch.unique), and the LDS-bitmap
  and hash-partition paths agree on i64_uniform_1e6;
* the three utf8 columns (5 % nulls): distinct count with the CAT +1 for
  nulls, top-50 by (count desc, key asc) and both Other rows, against a
  lexicographic sort of the strings as 16-byte keys.
Needs an MI355X with ~260 GB free.
"""

import pytest

import torch_ref

pytestmark = pytest.mark.gpu

ROWS = 10 ** 9


OTHER = ['***Other Values***', '***Other Values Distinct Count***']


def check_string_column(d, col, name, nrows):
    """One CAT string column of a describe() result vs torch: the strings as
    16-byte keys (torch_ref.short_string_keys), grouped by a lexicographic sort."""
    valid = torch_ref.valid_mask(col, nrows)
    n_valid = int(valid.sum().item())
    k0, k1 = torch_ref.short_string_keys(col, nrows, valid)
    del valid
    D, pairs, m = torch_ref.top_groups_pairs(k0, k1, 50)
    del k0, k1
    row = d['variables'].loc[name]
    assert row['type'] == 'CAT', (name, row['type'])
    assert int(row['count']) == m == n_valid, name
    assert int(row['n_missing']) == nrows - n_valid, name
    # CAT: countDistinct ignores nulls, then +1 when any value is missing (describe.py:169-170)
    assert int(row['distinct_count']) == D + (1 if nrows > n_valid else 0), (name, int(row['distinct_count']), D)
    want_idx = [torch_ref.key_pair_to_str(*kp) for kp, _ in pairs] + OTHER
    want_val = [c for _, c in pairs] + [m - sum(c for _, c in pairs), D - len(pairs)]
    fr = d['freq'][name]
    assert list(fr.index) == want_idx, (name, list(fr.index)[:5], want_idx[:5])
    assert [int(x) for x in fr.values] == want_val, name
    assert row['top'] == want_idx[0] and int(row['freq']) == want_val[0], name


def test_bench_table_properties_1e9():
    import torch
    import bench
    from spark_df_profiling import describe
    from spark_df_profiling.engine import Engine
    torch.cuda.empty_cache()
    dev = torch.device('cuda', 0)
    table = bench.make_c3_shard(ROWS, 0, 1, dev)
    raw = {}
    d = describe(table, raw=raw, plots=False)
    torch.cuda.empty_cache()
    v = d['variables']
    assert d['table']['n'] == ROWS
    cols = {c.name: c for c in table.columns}
    problems = []
    checked = 0
    for name, b in raw['columns'].items():
        col = cols[name]
        if 'numeric' not in b or v.loc[name, 'type'] == 'CORR':
            continue
        uniq = counts = None
        if not col.is_float:
            x = col.values[:ROWS]
            uniq, counts = torch.unique(x[torch_ref.valid_mask(col, ROWS)], sorted=True, return_counts=True)
        torch_ref.check_numeric(name, col, b['numeric'], v.loc[name], ROWS, uniq, counts, problems)
        del uniq, counts
        torch.cuda.empty_cache()
        checked += 1
    assert checked >= 11
    assert not problems, '\n'.join(problems[:40])
    # distinct counts of a float and the date column by torch.unique
    for name in ('f32_uniform', 'date'):
        c = cols[name]
        vals = c.values[:ROWS][torch_ref.valid_mask(c, ROWS)]
        want = int(torch.unique(vals).numel())
        del vals
        assert int(v.loc[name, 'distinct_count']) == want, name
    assert int(v.loc['i64_id', 'distinct_count']) == int(v.loc['i64_id', 'count'])
    # utf8 columns (CAT, 5 % nulls): exact distinct + the null quirk, top-50 by
    # (count desc, key asc) and both Other rows (describe.py:143,169-170,251-263)
    for name in ('str_card100', 'str_card1e5', 'str_card1e8'):
        check_string_column(d, cols[name], name, ROWS)
        torch.cuda.empty_cache()
    eng = Engine(device=dev)
    c = cols['i64_uniform_1e6']
    by_bitmap = int(v.loc['i64_uniform_1e6', 'distinct_count'])
    by_partition = eng.distinct_fixed(c, with_counts=False)['groups']
    assert by_bitmap == by_partition
    # the quantile fallback at full size: every window forced to miss, so every
    # rank of every column is re-collected from its key range and selected --
    # within the device budget, and the same quantiles as the checked run
    from spark_df_profiling import engine as engmod
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    saved = engmod.DEBUG_QUANTILE
    engmod.DEBUG_QUANTILE = 'miss'
    try:
        raw2 = {}
        d2 = describe(table, raw=raw2, plots=False)
    finally:
        engmod.DEBUG_QUANTILE = saved
    v2 = d2['variables']
    peak_extra = torch.cuda.max_memory_allocated(dev) - base
    used = [n for n, b in raw2['columns'].items() if 'numeric' in b and b['numeric'].fallback_used]
    assert len(used) >= 11, used
    for name in used:
        for q in ('5%', '25%', '50%', '75%', '95%'):
            assert float(v2.loc[name, q]) == float(v.loc[name, q]), (name, q)
    # one key range (<= 1e9 keys + 2x select workspace) at a time on top of the
    # describe() temporaries -- far inside the 288 GB device
    assert peak_extra < 140e9, peak_extra
    del table
    torch.cuda.empty_cache()
