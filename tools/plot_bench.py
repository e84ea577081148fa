"""Histogram image cost on this host: one process, then the pool on a C5-sized batch."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'spark-df-profiling_amd'))
import numpy as np
from spark_df_profiling import plot
from spark_df_profiling.utils import available_cpus
rng = np.random.default_rng(0)
items = [(rng.integers(0, 10 ** 6, 10), list(np.sort(rng.normal(size=10)) * (i + 1)), 0.1 * (i + 1)) for i in range(512)]
plot.render_pair(*items[0])
t = time.perf_counter()
for it in items[:64]:
    plot.render_pair(*it)
one = (time.perf_counter() - t) / 64 * 1e3
import cProfile, pstats, io
pr = cProfile.Profile(); pr.enable()
for it in items[:32]:
    plot.render_pair(*it)
pr.disable(); s = io.StringIO(); pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(8)
plot.start_pool()
t = time.perf_counter()
futs = plot.submit_batch(items)
res = [f.result() for f in futs]
pool = (time.perf_counter() - t) * 1e3
print('cpus', available_cpus(), 'pair %.2f ms one process; 512 pairs on the pool %.1f ms' % (one, pool))
print(s.getvalue()[:2500])
plot.shutdown_pool()
