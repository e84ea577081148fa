"""Vectorised mode of the oracle -- TEST INFRASTRUCTURE ONLY.

Same restatement as spark_describe.py (same functions, same formulas, same
reference line citations), with the row loops replaced by vectorised kernels so
that the BASELINE configurations can be checked at 1e6-1e7 rows:

* sums: numpy pairwise sums of 64 K-element chunks, the chunk partials added
  exactly (math.fsum) -- error <= ~16 eps * sum|x|, far inside the 1e-9
  relative bound of every statistic built from them (the exact mode is
  pinned against the known answers; tests/test_oracle_fast.py checks this mode
  against the exact one);
* order statistics: an introselect partition at the needed ranks (exact);
* countDistinct / groupBy counts: hash aggregation (pandas khash for numeric
  keys, Arrow's hash kernels otherwise) -- exact;
* top-50: only groups at or above the 50th largest count are sorted by key.

`describe(table, workers=N)` also runs the per-column work on N processes
(the multi-core CPU baseline of bench.py).  Start the pool with start_pool()
before the calling process initialises a GPU (spawned workers).
"""

from __future__ import annotations

from . import spark_describe as _sd

_POOL = None
_POOL_N = 0


def start_pool(workers):
    """A spawn-context process pool of `workers` processes (started once)."""
    global _POOL, _POOL_N
    if _POOL is None and workers > 1:
        import multiprocessing as mp
        import sys
        from concurrent.futures import ProcessPoolExecutor
        _POOL = ProcessPoolExecutor(max_workers=workers, mp_context=mp.get_context('spawn'))
        _POOL_N = workers
        # spawn re-imports the parent's __main__ in every child unless it cannot
        # find it; hide it while the workers start (they need only this package)
        main = sys.modules.get('__main__')
        saved = {a: getattr(main, a) for a in ('__file__', '__spec__') if main is not None and hasattr(main, a)}
        try:
            if '__file__' in saved:
                del main.__file__
            if '__spec__' in saved:
                main.__spec__ = None
            list(_POOL.map(_warm, range(2 * workers)))
        finally:
            for a, v in saved.items():
                setattr(main, a, v)
    return _POOL


def _warm(_):
    import pyarrow.compute  # noqa: F401
    return 0


def pool_workers():
    return _POOL_N if _POOL is not None else 1


def describe(table, bins=10, corr_reject=0.9, **kwargs):
    d, _ = _sd._describe_with_raw(table, bins, corr_reject, None, fast=True, pool=_POOL, **kwargs)
    return d


def profile_raw(table, bins=10, corr_reject=0.9, **kwargs):
    return _sd._describe_with_raw(table, bins, corr_reject, None, fast=True, pool=_POOL, **kwargs)
