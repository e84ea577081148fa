"""BASELINE.json configurations at their own sizes.

  C2  1e8 x 8 fp64                 vs the vectorised oracle (oracle/fast.py,
                                   pinned to the exact restatement by
                                   test_oracle_fast.py), every statistic
  C4  1e9 rows: int64 U[0,2^32) + 16-byte hex ids zipf(1.05) over 5e8 labels
                                   vs independent torch code on the device:
                                   distinct counts (torch.unique), top-50 by
                                   (count desc, key asc) and the two "Other"
                                   rows, every NUM statistic (torch_ref); the
                                   hex ids again with 5 % nulls (CAT +1 quirk)
  C5  1e7 x 512 fp32               the Pearson matrix vs a torch fp64 Gram of
                                   the same device data (1e-9), every NUM
                                   column's statistics vs torch_ref

Reference call sites: describe.py:143 (countDistinct), :193-223 (moments,
percentiles, mad, zeros, outliers), :251-263 (top-50 + Other rows), :38-63
(histogram), utils.py:20-36 (corr_matrix).  Needs an MI355X (~200 GB free).
"""

import numpy as np
import pytest

import datagen
import torch_ref

pytestmark = pytest.mark.gpu

OTHER = ['***Other Values***', '***Other Values Distinct Count***']


def test_c2_fp64_1e8_vs_oracle():
    import torch
    from test_gpu_configs import _check
    torch.cuda.empty_cache()
    t = datagen.c2_table(100_000_000)
    got, raw, want, want_raw = _check(t, t)
    v = got['variables']
    assert int(got['table']['n']) == 100_000_000
    assert abs(v.loc['shifted_1e9', 'variance'] - 1.0) < 1e-3
    del t
    torch.cuda.empty_cache()


def test_c4_high_cardinality_1e9():
    import torch
    import bench
    from spark_df_profiling import describe
    torch.cuda.empty_cache()
    dev = torch.device('cuda', 0)
    n = 10 ** 9
    table = bench.make_c4_shard(n, 0, 1, dev)
    raw = {}
    d = describe(table, raw=raw, plots=False)
    v = d['variables']
    assert d['table']['n'] == n
    # int64 U[0, 2^32): NUM (describe.py:158); countDistinct + every statistic
    c = table.column('u32_range_i64')
    uniq, counts = torch.unique(c.values, sorted=True, return_counts=True)
    problems = torch_ref.check_numeric('u32_range_i64', c, raw['columns']['u32_range_i64']['numeric'],
                                       v.loc['u32_range_i64'], n, uniq, counts)
    d_int = int(uniq.numel())
    del uniq, counts
    torch.cuda.empty_cache()
    assert d_int > 8 * 10 ** 8                              # near-unique, as the config intends
    # hex ids: CAT; exact distinct, top-50 (count desc, key asc) and the two Other rows
    keys = torch_ref.hex16_keys(table.column('hex_id'), n)
    D, pairs, rows = torch_ref.top_groups(keys, 50)
    del keys
    torch.cuda.empty_cache()
    row = v.loc['hex_id']
    assert row['type'] == 'CAT'
    assert int(row['count']) == rows == n
    assert int(row['distinct_count']) == D                  # no nulls: no +1 (describe.py:169-170)
    want_idx = [torch_ref.key_to_hex(k) for k, _ in pairs] + OTHER
    want_val = [cnt for _, cnt in pairs] + [n - sum(cnt for _, cnt in pairs), D - len(pairs)]
    fr = d['freq']['hex_id']
    assert list(fr.index) == want_idx
    assert [int(x) for x in fr.values] == want_val
    assert row['top'] == want_idx[0] and int(row['freq']) == want_val[0]
    assert not problems, '\n'.join(problems)
    # the same hex ids with 5 % nulls (a validity bitmap over the same strings):
    # the CAT distinct count gains the +1 for nulls (describe.py:169-170), the
    # top-50 and Other rows count only valid rows
    from spark_df_profiling.columns import DeviceColumn, DeviceTable
    from test_gpu_scale_1e9 import check_string_column
    hx = table.column('hex_id')
    hn = DeviceColumn('hex_id_nulls', 'string', n, 'bytes')
    hn.offsets, hn.data, hn.offset_width = hx.offsets, hx.data, hx.offset_width
    hn.validity = bench._validity(n, bench._gen(bench.SEED + 4003, dev), dev)
    t2 = DeviceTable([table.column('u32_range_i64'), hn], n)
    d2 = describe(t2, plots=False)
    del t2
    torch.cuda.empty_cache()
    check_string_column(d2, hn, 'hex_id_nulls', n)
    del table, hn, d2
    torch.cuda.empty_cache()


def test_c5_wide_pearson_1e7():
    import torch
    import bench
    from spark_df_profiling import describe
    torch.cuda.empty_cache()
    dev = torch.device('cuda', 0)
    n = 10 ** 7
    table = bench.make_c5_shard(n, 0, 1, dev)
    raw = {}
    d = describe(table, raw=raw, plots=False)
    v = d['variables']
    names = [c.name for c in table.columns]
    # Pearson (utils.py:20-36) vs a torch fp64 Gram of the centred columns
    X = torch.empty((n, len(names)), dtype=torch.float64, device=dev)
    for j, c in enumerate(table.columns):
        X[:, j] = c.values[:n].double()
    means = torch.tensor(torch_ref.fsum_cols(X), dtype=torch.float64, device=dev) / n
    X -= means[None, :]
    G = X.T @ X
    del X
    torch.cuda.empty_cache()
    dg = torch.sqrt(torch.diagonal(G))
    rho = (G / dg[:, None] / dg[None, :]).cpu().numpy()
    got = raw['corr'].to_numpy()
    assert got.shape == (512, 512)
    assert list(raw['corr'].index) == names
    err = np.abs(got - rho)
    assert np.all(err <= 1e-9 * np.abs(rho) + 1e-12), float(err.max())
    # CORR rejection (describe.py:89-100): the last earlier column with rho >= 0.9
    problems = []
    for i, x in enumerate(names):
        hits = [j for j in range(i) if rho[i, j] >= 0.9]
        row = v.loc[x]
        if hits:
            if row['type'] != 'CORR' or row['correlation_var'] != names[hits[-1]]:
                problems.append('%s: CORR with %s expected, got %s %s' % (x, names[hits[-1]], row['type'],
                                                                       row.get('correlation_var')))
        elif row['type'] == 'CORR':
            problems.append('%s: unexpected CORR' % x)
    # every column's statistics (CORR-rejected columns carry only the CORR keys)
    for c in table.columns:
        row = v.loc[c.name]
        if row['type'] == 'CORR':
            continue
        st = raw['columns'][c.name]['numeric']
        torch_ref.check_numeric(c.name, c, st, row, n, problems=problems)
        want_d = int(torch.unique(c.values[:n]).numel())       # no NaN, no nulls
        if int(row['distinct_count']) != want_d:
            problems.append('%s.distinct_count: %r vs %r' % (c.name, row['distinct_count'], want_d))
    assert not problems, '\n'.join(problems[:40])
    del table
    torch.cuda.empty_cache()
