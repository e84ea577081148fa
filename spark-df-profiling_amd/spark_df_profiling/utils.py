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
