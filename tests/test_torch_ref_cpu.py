"""The torch re-derivations used at BASELINE sizes (torch_ref.py) agree with
the oracle on CPU tensors: every NUM statistic of a mixed numeric table (NaN,
+-0.0, nulls, the 1e9-offset cancellation column, int8-int64) and the hex-id
top-k by (count desc, key asc)."""

import collections
import types

import numpy as np
import pyarrow as pa

import datagen
import torch_ref


def _device_table(t):
    from spark_df_profiling.columns import DeviceTable
    return DeviceTable.from_arrow(t, device='cpu', streamed=False)


def test_check_numeric_matches_oracle():
    from oracle import fast
    t = datagen.numeric_table(100_000).select(
        ['f64_norm', 'f64_shift', 'f64_logn', 'f64_nan_zero', 'f32_unif', 'i64_small', 'i64_wide', 'i64_zipf',
         'i16', 'i8'])
    want, raw = fast.profile_raw(t)
    problems = []
    checked = 0
    for c in _device_table(t).columns:
        row = want['variables'].loc[c.name]
        if row['type'] != 'NUM':
            continue
        r = raw['columns'][c.name]
        st = types.SimpleNamespace(edges=r['hist']['edges'], hist_counts=r['hist']['counts'],
                                   thresholds=r['thresholds'])
        torch_ref.check_numeric(c.name, c, st, row, t.num_rows, problems=problems)
        checked += 1
    assert checked >= 8
    assert not problems, '\n'.join(problems)


def test_check_numeric_flags_a_wrong_value():
    from oracle import fast
    t = datagen.numeric_table(20_000).select(['f64_norm', 'i64_small'])
    want, raw = fast.profile_raw(t)
    for c in _device_table(t).columns:
        row = want['variables'].loc[c.name].copy()
        row['mean'] = float(row['mean']) * (1 + 1e-7)
        row['25%'] = float(row['25%']) + 1.0
        r = raw['columns'][c.name]
        st = types.SimpleNamespace(edges=r['hist']['edges'], hist_counts=np.asarray(r['hist']['counts']) + 1,
                                   thresholds=r['thresholds'])
        problems = torch_ref.check_numeric(c.name, c, st, row, t.num_rows)
        keys = {p.split(':')[0].split('.', 1)[1] for p in problems}
        assert {'mean', 'histogram'} <= keys, problems
        assert any('quantile' in k for k in keys), problems


def test_hex_top_groups():
    lab = (np.arange(5000) * 7919) % 113
    strs = datagen.hex16_strings(datagen.mix64_np(lab))
    col = _device_table(pa.table({'h': strs})).columns[0]
    keys = torch_ref.hex16_keys(col, 5000)
    D, pairs, rows = torch_ref.top_groups(keys, 50)
    cc = collections.Counter(strs.to_pylist())
    want = sorted(cc.items(), key=lambda kv: (-kv[1], kv[0]))[:50]
    assert D == len(cc) and rows == 5000
    assert [(torch_ref.key_to_hex(k), c) for k, c in pairs] == want


def test_short_string_keys_and_pair_groups():
    """The 1e9-row string checker (torch_ref.short_string_keys +
    top_groups_pairs) against a plain Python count on ragged strings with
    nulls, ties and prefixes of one another."""
    import torch
    rng = np.random.default_rng(5)
    alphabet = [b'a', b'b', b'ab', b'abc', b'abcdefgh', b'abcdefghi', b'zzzzzzzzzzzzzzzz', b'q', b'0123456789abcdef']
    vals = [alphabet[i] if rng.random() > 0.1 else None for i in rng.integers(0, len(alphabet), 3000)]
    data = b''.join(v for v in vals if v) + b'\0' * 16
    offs = [0]
    for v in vals:
        offs.append(offs[-1] + (len(v) if v else 0))
    col = types.SimpleNamespace(data=torch.tensor(list(data), dtype=torch.uint8),
                                offsets=torch.tensor(offs, dtype=torch.int64), fixed_width=0)
    valid = torch.tensor([v is not None for v in vals])
    k0, k1 = torch_ref.short_string_keys(col, len(vals), valid, chunk=1000)
    D, pairs, m = torch_ref.top_groups_pairs(k0, k1, 4)
    cnt = collections.Counter(v for v in vals if v is not None)
    want = sorted(cnt.items(), key=lambda kv: (-kv[1], kv[0]))[:4]
    assert (D, m) == (len(cnt), sum(cnt.values()))
    assert [(torch_ref.key_pair_to_str(*kp).encode(), c) for kp, c in pairs] == want
