"""The shifted Gram product behind corr_matrix (utils.py:20-36) on every tile
width the kernel has (16 / 32 / 64 columns per tile, diagonal and off-diagonal
tiles), with mixed dtypes, nulls and NaN (listwise deletion, utils.py:27),
against numpy float64 (tables of <= 16 columns: gram16_kernel).  Tolerance: 1e-12 relative to sum |x - K|^2 per entry
(the kernel's summation order differs from numpy's; both are fp64)."""

import numpy as np
import pyarrow as pa
import pytest

pytestmark = pytest.mark.gpu

DTYPES = [np.float64, np.int64, np.float32, np.int32, np.int16, np.uint8, np.uint32, np.float64]


def _table(n, ncols, seed, dtypes=DTYPES):
    g = np.random.default_rng(seed)
    cols, host = {}, []
    base = g.standard_normal(n)
    for c in range(ncols):
        dt = dtypes[c % len(dtypes)]
        x = 40 * (0.5 * base + g.standard_normal(n)) + (c % 5) * 7
        if np.issubdtype(dt, np.unsignedinteger):
            x = np.clip(np.abs(x), 0, 250)
        v = x.astype(dt)
        mask = g.random(n) < (0.02 if c % 3 == 0 else 0.0)
        if dt == np.float64 and c % 4 == 0:
            v[g.random(n) < 0.01] = np.nan
        cols['c%03d' % c] = pa.array(v, mask=mask)
        xd = v.astype(np.float64)
        xd[mask] = np.nan
        host.append(xd)
    return pa.table(cols), np.stack(host, axis=1)


# > 64 columns take the wide kernel (128-column tiles): diagonal and
# off-diagonal tiles x {all f32, all f64, mixed} staging paths, padding
# columns of a partial last tile, chunks with a ragged tail (n % 4 != 0),
# several row chunks per tile.
WIDE = [(2053, 70, None), (20011, 200, None), (40000, 160, 'f32'), (9999, 130, 'f32'), (30002, 257, 'f64'),
        (7, 129, 'f64'), (3, 300, None)]


# <= 16 columns take gram16_kernel (256-row k-steps, one column per wave while
# staging): several chunks with a ragged last k-step, every dtype, 1-16 columns
NARROW = [(5003, 12, None), (1, 3, None), (300_001, 16, None), (257, 5, None), (70_003, 16, 'f64'),
          (1_048_579, 9, None), (4, 1, None)]


@pytest.mark.parametrize('n,ncols,kind', NARROW + [(4099, 21, None), (3001, 40, None), (37, 17, None)] + WIDE)
def test_gram_matches_numpy(n, ncols, kind):
    import torch
    from spark_df_profiling.columns import DeviceTable
    from spark_df_profiling.engine import Engine
    dtypes = {None: DTYPES, 'f32': [np.float32], 'f64': [np.float64]}[kind]
    tab, X = _table(n, ncols, seed=n + ncols, dtypes=dtypes)
    dt = DeviceTable.from_arrow(tab, torch.device('cuda'))
    cols = [dt.column(c) for c in tab.column_names]
    keep = ~np.isnan(X).any(axis=1)
    K = np.array([np.nanmean(X[:, j]) if np.isfinite(X[:, j]).any() else 0.0 for j in range(ncols)])
    G, s, nk = Engine().gram(cols, K.tolist(), [True] * ncols)
    Y = X[keep] - K
    want_G = Y.T @ Y
    scale = np.sqrt(np.outer(np.diag(want_G), np.diag(want_G))) + 1e-300
    assert nk == keep.sum()
    assert np.all(np.abs(G - want_G) <= 1e-12 * scale + 1e-300)
    assert np.allclose(s, Y.sum(axis=0), rtol=1e-12, atol=1e-9 * np.sqrt(np.diag(want_G)).max() + 1e-300)
