import sys, os
sys.path.insert(0, 'tests'); sys.path.insert(0, 'spark-df-profiling_amd'); sys.path.insert(0, '.')
import datagen
from spark_df_profiling.columns import DeviceTable
from spark_df_profiling.engine import Engine, PROBS, spark_percentile_approx_rank
import math
t = datagen.numeric_table(200_003)
dt = DeviceTable.from_arrow(t)
e = Engine()
for c in dt.columns:
    p1, plan, ci = e.numeric_pass1(c)
    n = p1['count']
    print(c.name, 'n', n, 'nw', plan.n_windows, 'ns', plan.n_sample, 'grid', ci['grid'], 'cap', ci['cap'], 'ovf', p1['w_overflow'])
    for w in range(plan.n_windows):
        size = p1['w_eq_lo'][w] + p1['w_in'][w] + p1['w_eq_hi'][w]
        below = n - p1['w_gt'][w] - size
        print('   w', w, 'lo', hex(plan.lo[w]), 'hi', hex(plan.hi[w]), 'in_s', plan.in_sample[w], 'below', below, 'size', size, 'eqlo', p1['w_eq_lo'][w], 'in', p1['w_in'][w], 'eqhi', p1['w_eq_hi'][w], 'gt', p1['w_gt'][w])
    ranks = [spark_percentile_approx_rank(n, p) - 1 if c.is_float else math.floor((n - 1) * p) for p in PROBS]
    print('   ranks', ranks)
