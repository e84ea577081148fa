"""The Spark 2.x percentile_approx restatement (oracle/gk.py) on the CPU:
small cases worked by hand from QuantileSummaries' rules, and Spark's
documented guarantee -- the returned element's rank lies
within ceil(N / accuracy) of ceil(p N) -- on multi-batch, multi-partition
inputs.  Parity with Spark itself is unpinned (no Spark here)."""

import math

import numpy as np

from oracle import gk

PROBS = [0.05, 0.25, 0.5, 0.75, 0.95]


def _rank_ok(values, got, p, accuracy):
    s = np.sort(np.asarray(values, dtype=np.float64))
    n = s.size
    lo = np.searchsorted(s, got, 'left') + 1          # 1-based ranks the value occupies
    hi = np.searchsorted(s, got, 'right')
    target = math.ceil(p * n)
    err = math.ceil(n / accuracy)
    return lo - err <= target <= hi + err


def test_tiny_partition_is_exact_order_statistic():
    # fewer than 5000 values: every delta is 0 and nothing merges; sample i
    # (0-based, i >= 1) has minRank i, so the query returns the first i with
    # i + 1 >= ceil(pN): the element of rank ceil(pN) (rank 3 of 5 for p = 0.5)
    vals = [5.0, 1.0, 4.0, 2.0, 3.0]
    s = gk.partition_digest(vals, 1e-4)
    assert [t[0] for t in s.sampled] == [1.0, 2.0, 3.0, 4.0, 5.0]
    assert all(t[1] == 1 and t[2] == 0 for t in s.sampled)
    assert gk.percentile_approx([vals], [0.0, 0.5, 1.0]) == [1.0, 3.0, 5.0]


def test_negative_zero_sorts_first():
    s = gk.partition_digest([0.0, -0.0, 1.0], 1e-4)
    v = [t[0] for t in s.sampled]
    assert math.copysign(1.0, v[0]) == -1.0 and math.copysign(1.0, v[1]) == 1.0


def test_rank_window_multi_batch_partitions():
    rng = np.random.default_rng(20261017)
    vals = rng.standard_normal(130_001)
    parts = gk.split_rows(vals, None, 3)
    got = gk.percentile_approx(parts, PROBS)
    for p, g in zip(PROBS, got):
        assert _rank_ok(vals, g, p, 10000), (p, g)


def test_rank_window_duplicates_and_low_accuracy():
    rng = np.random.default_rng(7)
    vals = rng.integers(0, 50, 60_000).astype(np.float64)
    parts = gk.split_rows(vals, None, 2)
    for acc in (100, 10000):
        got = gk.percentile_approx(parts, PROBS, accuracy=acc)
        for p, g in zip(PROBS, got):
            assert _rank_ok(vals, g, p, acc), (acc, p, g)


def test_empty_partitions_are_skipped():
    a = gk.percentile_approx([[], [3.0, 1.0, 2.0], []], [0.5])
    b = gk.percentile_approx([[3.0, 1.0, 2.0]], [0.5])
    assert a == b


def test_query_rank_saturates_like_scala_toint():
    # QuantileSummaries.query: rank = math.ceil(q * count).toInt, which
    # saturates at Int.MaxValue once q * count >= 2^31 (a row-sharded table of
    # ~2.3e9 values at q = 0.95).  Interior samples at minRank 2^31 - 2 and
    # 3e9 - 2 (target error 3): the saturated rank matches the first; the
    # unbounded rank 2.85e9 matches none and falls through to the maximum.
    count = 3 * 10 ** 9
    m = gk.INT_MAX
    sampled = [(0.0, 1, 0), (1.0, m - 1, 0), (2.0, count - m - 1, 0), (3.0, 1, 0)]
    s = gk.Summary(1e-9, sampled, count)
    assert s.query(0.95) == 1.0          # rank min(ceil(2.85e9), 2^31 - 1) = 2^31 - 1 = minRank of 1.0
    assert s.query(0.5) == 3.0           # ceil(1.5e9) < 2^31 - 1 matches no interior sample: the maximum
