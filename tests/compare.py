"""Compare a describe() result with the oracle's, cell by cell.

Tolerances (BASELINE.json north_star): counts, distinct counts, n_zeros,
outlier counts, top-N and frequency tables bit-exact; quantiles exact (the
engine returns the exact order statistic the oracle defines); fp64 moments and
ratios within 1e-9 relative, with an absolute floor of 1e-12 x scale for
statistics that can sit at 0 (skewness of symmetric data, cv near zero mean).
"""

import datetime
import decimal
import math

import numpy as np
import pandas as pd

REL = 1e-9
SKIP = {'histogram', 'mini_histogram'}


def _isnan(v):
    return isinstance(v, (float, np.floating)) and math.isnan(v)


def close(a, b, rel=REL, floor=1e-12):
    a, b = float(a), float(b)
    if math.isnan(a) or math.isnan(b):
        return math.isnan(a) and math.isnan(b)
    if math.isinf(a) or math.isinf(b):
        return a == b
    return abs(a - b) <= rel * max(abs(a), abs(b)) + floor


def same_value(key, a, b):
    if key in SKIP:
        return True
    if _isnan(a) or _isnan(b) or a is None or b is None:
        return (_isnan(a) or a is None) and (_isnan(b) or b is None)
    if isinstance(a, pd.Series) or isinstance(b, pd.Series):
        return series_equal(a, b)
    if isinstance(a, (str, bytes, bool, np.bool_, datetime.date, datetime.timedelta, decimal.Decimal,
                      pd.Timestamp)):
        return a == b
    if isinstance(a, (int, np.integer)) and isinstance(b, (int, np.integer)):
        return int(a) == int(b)
    if isinstance(a, (float, np.floating, int, np.integer)):
        if key in ('5%', '25%', '50%', '75%', '95%', 'min', 'max', 'range', 'iqr'):
            # order statistics are elements (or Spark's interpolation of two)
            # and their differences: the engine returns the same values
            return float(a) == float(b)
        scale_floor = 1e-12 if key in ('skewness', 'kurtosis', 'cv', 'correlation', 'accuracy_idx') else 0.0
        return close(a, b, floor=scale_floor)
    return a == b


def series_equal(a, b):
    if not (isinstance(a, pd.Series) and isinstance(b, pd.Series)):
        return False
    if len(a) != len(b):
        return False
    for (ka, va), (kb, vb) in zip(a.items(), b.items()):
        if not same_value('key', ka, kb) or not same_value('vc', va, vb):
            return False
    return True


def assert_describe_equal(got, want):
    assert set(got.keys()) == {'table', 'variables', 'freq'}
    problems = []
    gt, wt = got['table'], want['table']
    if set(gt) != set(wt):
        problems.append('table keys %s vs %s' % (sorted(gt), sorted(wt)))
    for k in wt:
        if k in gt and not same_value(k, gt[k], wt[k]):
            problems.append('table[%s]: %r vs %r' % (k, gt[k], wt[k]))
    gv, wv = got['variables'], want['variables']
    integral = set(wv.attrs.get('integral_num', ()))
    if list(gv.index) != list(wv.index):
        problems.append('variables index %s vs %s' % (list(gv.index), list(wv.index)))
    if set(gv.columns) != set(wv.columns):
        problems.append('variables columns differ: +%s -%s' % (set(gv.columns) - set(wv.columns),
                                                               set(wv.columns) - set(gv.columns)))
    for name in wv.index:
        if name not in gv.index:
            continue
        for k in wv.columns:
            if k not in gv.columns:
                continue
            a, b = gv.loc[name, k], wv.loc[name, k]
            if k == 'mad' and not _isnan(b) and b is not None:
                # mad inherits the mean's last-ulp rounding: |d mad / d mean| <= 1
                m = float(wv.loc[name, 'mean'])
                if abs(float(a) - float(b)) <= REL * abs(float(b)) + 4 * np.spacing(abs(m)):
                    continue
            if k == 'sum' and name in integral:
                # float(two's-complement int64 sum): describe.py:200 Sum of a
                # LongType, upcast to double by .ix[0] at :209 -- exact
                if not (float(a) == float(b)):
                    problems.append('%s.sum (integral, exact): %r vs %r' % (name, a, b))
                continue
            if not same_value(k, a, b):
                problems.append('%s.%s: %r vs %r' % (name, k, a, b))
    if set(got['freq']) != set(want['freq']):
        problems.append('freq keys %s vs %s' % (sorted(got['freq']), sorted(want['freq'])))
    for k in want['freq']:
        if k in got['freq'] and not series_equal(got['freq'][k], want['freq'][k]):
            problems.append('freq[%s]:\n%s\nvs\n%s' % (k, got['freq'][k], want['freq'][k]))
    assert not problems, '\n'.join(problems[:40])
