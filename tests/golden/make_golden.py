"""Writes known_answers.json: Spark-semantics known answers for the reference's
own legacy test data (/root/reference/spark_df_profiling/tests.py.old.py:23-37).

The values are literals, not oracle output: they are the legacy test's expected
values that hold under Spark semantics (tests.py.old.py:58-76, re-derived in
SURVEY.md Appendix D by hand/recomputation), plus the Spark-specific ones
Appendix D lists (population skewness/kurtosis, Spark percentile interpolation,
countDistinct ignoring nulls, accumulated histogram edges).  The oracle is
pinned against this file by tests/test_oracle_golden.py.

Column x is typed bigint with a null (Spark's view of the int column); the
distinct count is 6 (countDistinct ignores the null; the legacy 7 counted it).
"""

import json
import os

KNOWN = {
    'table': {'n': 9, 'nvar': 7, 'total_missing': 0.063492063492063489,
              'NUM': 2, 'CAT': 1, 'CONST': 2, 'DATE': 1, 'UNIQUE': 1, 'CORR': 0},
    'x': {  # tests.py.old.py:58-65 (Spark-valid subset) + SURVEY.md App. D
        'count': 8, 'n_missing': 1, 'distinct_count': 6, 'mean': 13.375, 'variance': 561.125,
        'std': 23.688077169749342, 'sum': 107.0, 'mad': 18.71875, 'min': -10.0, 'max': 50.0,
        'range': 60.0, 'iqr': 24.5, 'cv': 1.771071190261633, 'p_zeros': 0.2222222222222222,
        'n_zeros': 2, 'high_idx': 0, 'low_idx': 0, 'type': 'NUM',
        '5%': -7.5499999999999989, '25%': -0.75, '50%': 2.5, '75%': 23.75, '95%': 50.0,
        'skewness': 0.8700654233008702, 'kurtosis': -0.9061564710904944,
        'hist_edges': [-10.0, -4.0, 2.0, 8.0, 14.0, 20.0, 26.0, 32.0, 38.0, 44.0],
        'hist_counts': [1, 3, 1, 0, 1, 0, 0, 0, 0, 2],
    },
    'y': {  # tests.py.old.py:66-76 (Spark-valid subset) + App. D
        'count': 8, 'n_missing': 1, 'mean': 491.17436504331249, 'variance': 1179686.0311895239,
        'std': 1086.1335236468506, 'sum': 3929.3949203464999, 'mad': 698.45081747834365,
        'min': -3.1415926535000001, 'max': 3122.0, 'range': 3125.1415926535001,
        'cv': 2.2112992878833846, 'p_zeros': 0.0, 'type': 'NUM',
        'skewness': 2.097192909339155, 'kurtosis': 2.654350961293982,
        'hist_counts': [6, 0, 1, 0, 0, 0, 0, 0, 0, 1],
    },
    'cat': {'count': 8, 'distinct_count': 7, 'mode': 'c', 'top': 'c', 'freq': 3, 'type': 'CAT',
            'n_missing': 1},
    's1': {'type': 'CONST', 'mode': 1.0, 'count': 9, 'distinct_count': 1},
    's2': {'type': 'CONST', 'mode': 'some constant text $ % value {obj} ', 'count': 9},
    'id': {'type': 'UNIQUE', 'count': 9, 'distinct_count': 9, 'is_unique': True, 'p_unique': 1.0},
    'somedate': {'type': 'DATE', 'count': 8, 'n_missing': 1, 'distinct_count': 5,
                 'min': '1898-01-02 00:00:00', 'max': '2022-01-01 13:57:00'},
}

if __name__ == '__main__':
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'known_answers.json')
    with open(out, 'w') as f:
        json.dump(KNOWN, f, indent=1, sort_keys=True)
    print('wrote', out)
