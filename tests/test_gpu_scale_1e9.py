"""The bench table itself (1e9 rows x 16 columns, bench.make_c3_shard) profiled
once, with size-independent properties checked at full size.  The exact
integer outputs are re-derived by independent torch code on the same device
(comparisons and sorts, no libsdp):

* histogram bins: #(x >= e_j) differences over the valid rows, exactly;
* n_zeros and the high/low outlier counts against the same thresholds;
* every float quantile is the element of rank ceil(pN): #(x < q) < r <= #(x <= q);
* count / n_missing from the validity bitmaps;
* distinct counts of i64_id (== count), f32_uniform and date (torch.unique),
  and the LDS-bitmap and hash-partition paths agree on i64_uniform_1e6;
* quantiles are monotone and lie in [min, max]; mean within [min, max].
Needs an MI355X with ~260 GB free.
"""

import math

import pytest

pytestmark = pytest.mark.gpu

ROWS = 10 ** 9


def _valid(col, n):
    import torch
    if col.validity is None:
        return torch.ones(n, dtype=torch.bool, device=col.values.device)
    bits = col.validity[:(n + 7) // 8]
    shifts = torch.arange(8, dtype=torch.uint8, device=bits.device)
    v = ((bits[:, None] >> shifts[None, :]) & 1).bool().reshape(-1)[:n]
    return v


def test_bench_table_properties_1e9():
    import torch
    import bench
    from spark_df_profiling import describe
    from spark_df_profiling.engine import Engine, spark_percentile_approx_rank
    torch.cuda.empty_cache()
    dev = torch.device('cuda', 0)
    table = bench.make_c3_shard(ROWS, 0, 1, dev)
    raw = {}
    d = describe(table, raw=raw, plots=False)
    v = d['variables']
    assert d['table']['n'] == ROWS
    cols = {c.name: c for c in table.columns}
    for name, b in raw['columns'].items():
        col = cols[name]
        if 'numeric' not in b:
            continue
        st = b['numeric']
        if v.loc[name, 'type'] == 'CORR':
            continue
        valid = _valid(col, ROWS)
        x = col.values[:ROWS]
        xd = x.double()
        ok = valid & ~torch.isnan(xd) if col.is_float else valid
        cnt = int(ok.sum().item())
        assert st.count == cnt and int(v.loc[name, 'count']) == cnt, name
        assert int(v.loc[name, 'n_missing']) == ROWS - cnt, name
        xs = xd[ok]
        del xd
        # histogram: CASE-WHEN bins from the host-accumulated edges
        ge = [int((xs >= float(e)).sum().item()) for e in st.edges]
        want = [ge[j] - ge[j + 1] for j in range(len(ge) - 1)] + [ge[-1]]
        assert list(map(int, st.hist_counts)) == want, name
        assert sum(want) == cnt, name
        # zeros and outliers (no NaN in this table)
        assert st.n_zero == int((xs == 0.0).sum().item()), name
        hi_t, lo_t = st.thresholds
        assert st.high_idx == int((xs > hi_t).sum().item()), name
        assert st.low_idx == int((xs < lo_t).sum().item()), name
        # quantiles: monotone, within [min, max], float ones of exact rank
        qs = [st.quantiles[p] for p in (0.05, 0.25, 0.5, 0.75, 0.95)]
        assert qs == sorted(qs) and st.min <= qs[0] and qs[-1] <= st.max, name
        assert st.min <= st.mean <= st.max, name
        assert float(xs.min().item()) == st.min and float(xs.max().item()) == st.max, name
        if col.is_float:
            for p, q in st.quantiles.items():
                r = spark_percentile_approx_rank(cnt, p)
                below = int((xs < q).sum().item())
                le = int((xs <= q).sum().item())
                assert below < r <= le, (name, p)
        del xs, ok, valid
    # distinct counts by torch.unique on a few columns
    eng = Engine(device=dev)
    idc = cols['i64_id']
    assert int(v.loc['i64_id', 'distinct_count']) == int(_valid(idc, ROWS).sum().item())
    for name in ('f32_uniform', 'date'):
        c = cols[name]
        vals = c.values[:ROWS][_valid(c, ROWS)]
        want = int(torch.unique(vals).numel())
        del vals
        assert int(v.loc[name, 'distinct_count']) == want, name
    c = cols['i64_uniform_1e6']
    by_bitmap = int(v.loc['i64_uniform_1e6', 'distinct_count'])
    by_partition = eng.distinct_fixed(c, with_counts=False)['groups']
    assert by_bitmap == by_partition
    torch.cuda.empty_cache()
