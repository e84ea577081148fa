"""A C host (examples/c_caller/sdp_profile.c: gcc + the HIP runtime, no Python
or torch) computes every statistic group of describe() through the coarse
C-ABI entries of include/sdp.h alone -- sdp_quantiles, sdp_pass1, sdp_pass2,
sdp_hash_distinct_count, sdp_value_counts_topk, sdp_minmax_int, sdp_gram_f64
 -- and its output is compared with the oracle on the same
table: counts, distinct counts, histogram bins, zeros, outlier counts,
quantiles and top-50 + Other rows bit-exact; moments, mad and the Pearson
matrix within 1e-9 relative (tests/compare.py).  Reference call sites:
describe.py:143,144,193-223,233,251-263, utils.py:20-36.  Needs an MI355X.
"""

import datetime
import json
import math
import os
import subprocess

import numpy as np
import pyarrow as pa
import pytest

import datagen
from compare import close

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, 'examples', 'c_caller', 'sdp_profile')
DTYPE = {'float64': 6, 'float32': 5, 'int64': 4, 'int32': 3, 'int16': 2, 'int8': 1, 'uint32': 9}


def _table(n, seed):
    g = datagen.rng(seed)
    cols, spec = {}, []
    f = g.standard_normal(n)
    f[g.random(n) < 0.01] = np.nan
    f[g.random(n) < 0.02] = 0.0
    vals = {'f64_nan': f, 'f64_shift': 1e9 + g.standard_normal(n), 'f32_u': g.random(n).astype(np.float32),
            'i64_wide': g.integers(-2 ** 40, 2 ** 40, n), 'i64_zipf': np.minimum(g.zipf(1.3, n), 10 ** 6).astype(np.int64),
            'i32_small': g.integers(-500, 500, n).astype(np.int32)}
    for name, v in vals.items():
        valid = g.random(n) >= 0.05
        cols[name] = pa.array(v, mask=~valid)
        spec.append(('num', name, v, valid))
    days = g.integers(-100000, 50000, n).astype(np.int32)
    dvalid = g.random(n) >= 0.03
    cols['day'] = pa.array(days, mask=~dvalid).cast(pa.date32())
    spec.append(('date', 'day', days, dvalid))
    labels = np.minimum(g.zipf(1.2, n), 5000)
    strs = np.array(['k%x_%s' % (l, 'z' * (l % 19)) for l in labels], dtype=object)
    svalid = g.random(n) >= 0.08
    cols['label'] = pa.array(list(strs), mask=~svalid)
    spec.append(('str', 'label', strs, svalid))
    return pa.table(cols), spec


def _write(tmp, spec, n):
    lines = []
    for kind, name, v, valid in spec:
        vb = os.path.join(tmp, name + '.valid')
        np.packbits(valid, bitorder='little').tofile(vb)
        if kind == 'str':
            b = [s.encode() if ok else b'' for s, ok in zip(v, valid)]
            offs = np.zeros(n + 1, dtype=np.int64)
            np.cumsum([len(x) for x in b], out=offs[1:])
            of, df = os.path.join(tmp, name + '.offs'), os.path.join(tmp, name + '.data')
            offs.tofile(of)
            with open(df, 'wb') as fh:
                fh.write(b''.join(b))
            lines.append('str %s %d %s %s %s' % (name, n, of, df, vb))
        else:
            path = os.path.join(tmp, name + '.bin')
            np.ascontiguousarray(v).tofile(path)
            if kind == 'date':
                lines.append('date %s %d %s %s' % (name, n, path, vb))
            else:
                lines.append('num %s %d %d %s %s' % (name, DTYPE[str(v.dtype)], n, path, vb))
    man = os.path.join(tmp, 'manifest.txt')
    with open(man, 'w') as fh:
        fh.write('\n'.join(lines) + '\n')
    return man


OTHER = ['***Other Values***', '***Other Values Distinct Count***']


@pytest.mark.parametrize('n,seed', [(200_003, 71), (5_001, 73)])      # partitioned and global-table paths
def test_c_host_matches_oracle(tmp_path, n, seed):
    import oracle
    assert os.path.exists(EXE), 'build examples/c_caller first (__graft_entry__.build())'
    table, spec = _table(n, seed)
    man = _write(str(tmp_path), spec, n)
    out = subprocess.run([EXE, man], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    got = json.loads(out.stdout)
    want, raw = oracle.profile_raw(table)
    v = want['variables']
    assert list(got['columns']) == [x[1] for x in spec]
    # both grouping paths are exercised: partitions at >= 64 K rows, the global table below
    path = 1 if n >= (1 << 16) else 2
    assert got['columns']['label']['path'] == path and got['columns']['i64_wide']['distinct_path'] == path
    assert got['columns']['i32_small']['distinct_path'] == 0                  # LDS bitmap (range <= 2^20)
    bad = []
    for name, c in got['columns'].items():
        row = v.loc[name]
        if c['kind'] == 'num':
            for key in ('count', 'n_zeros', 'high_idx', 'low_idx', 'distinct'):
                w = int(row['distinct_count' if key == 'distinct' else key])
                if int(c[key]) != w:
                    bad.append((name, key, c[key], w))
            for key in ('min', 'max', 'mean', 'variance', 'std', 'skewness', 'kurtosis', 'mad', 'sum'):
                if not close(c[key], float(row[key])):
                    bad.append((name, key, c[key], float(row[key])))
            for q, p in zip(c['quantiles'], ('5%', '25%', '50%', '75%', '95%')):
                if float(q) != float(row[p]):
                    bad.append((name, p, q, float(row[p])))
            if [int(x) for x in c['hist']] != [int(x) for x in raw['columns'][name]['hist']['counts']]:
                bad.append((name, 'hist', c['hist'], list(raw['columns'][name]['hist']['counts'])))
        elif c['kind'] == 'date':
            epoch = datetime.date(1970, 1, 1)
            if (int(c['count']), int(c['distinct'])) != (int(row['count']), int(row['distinct_count'])):
                bad.append((name, 'count/distinct', c['count'], c['distinct']))
            if (c['min'], c['max']) != ((row['min'] - epoch).days, (row['max'] - epoch).days):
                bad.append((name, 'min/max', c['min'], c['max']))
        else:
            # CAT: countDistinct + 1 for nulls (describe.py:169-170); top-50 + Other rows (:259-268)
            if int(c['groups']) + 1 != int(row['distinct_count']) or int(c['distinct']) != int(c['groups']):
                bad.append((name, 'distinct', c['groups'], c['distinct'], row['distinct_count']))
            fr = want['freq'][name]
            top = [(s, int(k)) for s, k in c['top']]
            w_top = list(zip(list(fr.index)[:-2], [int(x) for x in fr.values][:-2]))
            if top != w_top:
                bad.append((name, 'top50', top[:5], w_top[:5]))
            other = [int(c['rows']) - sum(k for _, k in top), int(c['groups']) - len(top)]
            if list(fr.index)[-2:] != OTHER or [int(x) for x in fr.values][-2:] != other:
                bad.append((name, 'other', other, list(fr.values)[-2:]))
    # Pearson of every numeric column, listwise deletion (utils.py:27-31)
    rc = raw['corr']
    names = got['corr_names']
    C = np.array(got['corr'], dtype=np.float64).reshape(len(names), len(names))
    W = rc.loc[names, names].to_numpy()
    for i in range(len(names)):
        for j in range(len(names)):
            if not (close(C[i, j], W[i, j]) or (math.isnan(C[i, j]) and math.isnan(W[i, j]))):
                bad.append(('corr', names[i], names[j], C[i, j], W[i, j]))
    assert not bad, bad[:20]
