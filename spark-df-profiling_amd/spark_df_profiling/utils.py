"""Helpers shared by describe(): percentile labels and the Pearson matrix.

`pretty_name` follows /root/reference/spark_df_profiling/utils.py:7-12 (the
labels '5%', '25%', ... are keys of the output).  `corr_from_gram` turns the
GPU Gram product into the matrix the reference builds with C^2 Spark
`df.stat.corr` jobs (utils.py:20-36, Spark CovarianceCounter: rho =
Ck / sqrt(MkX * MkY)).
"""

import numpy as np


def pretty_name(x):
    pct = x * 100
    if pct == int(pct):
        return '%.0f%%' % pct
    return '%.1f%%' % pct


def corr_from_gram(G, s, n):
    """rho from the shifted Gram G = sum (x-K)(x-K)^T, s = sum (x-K), n rows.

    C = G - s s^T / n are the co-moments about the kept rows' means (the shift
    K cancels exactly in exact arithmetic; it keeps G well conditioned)."""
    G = np.asarray(G, dtype=np.float64)
    s = np.asarray(s, dtype=np.float64)
    if n <= 0:
        return np.full(G.shape, np.nan)
    C = G - np.outer(s, s) / n
    d = np.diag(C).copy()
    with np.errstate(all='ignore'):
        rho = C / np.sqrt(np.outer(d, d))
    return rho


def available_cpus():
    """(CPUs this process may run on, how that was decided): the affinity mask,
    bounded by the cgroup CPU quota when one is set -- os.cpu_count() reports
    the whole machine (256 on the GPU box, whose job quota is 16)."""
    import math
    import os
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = os.cpu_count() or 1
    quota = None
    try:                                            # cgroup v2
        with open('/sys/fs/cgroup/cpu.max') as fh:
            q, per = fh.read().split()[:2]
        if q != 'max':
            quota = max(1, math.ceil(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if quota is None:                               # cgroup v1
        try:
            with open('/sys/fs/cgroup/cpu/cpu.cfs_quota_us') as fh:
                q = int(fh.read())
            with open('/sys/fs/cgroup/cpu/cpu.cfs_period_us') as fh:
                per = int(fh.read())
            if q > 0:
                quota = max(1, math.ceil(q / per))
        except (OSError, ValueError):
            pass
    if quota is not None and quota < allowed:
        return quota, 'cgroup cpu quota'
    return allowed, 'affinity mask'
