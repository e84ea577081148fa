"""The partition mixer's host-side inverse (engine.inv_mix64) against a plain
restatement of mix64 (sdp_common.h: fold, odd multiply, fold): fixed keys
recovered from their records must be the keys (top-k values of CAT and
NUM value counts).  CPU only."""

import numpy as np

from spark_df_profiling.engine import inv_mix64, U64


def mix64(x):
    x ^= x >> 32
    x = (x * 0xD6E8FEB86659FD93) & U64
    return x ^ (x >> 32)


def test_inverse_round_trips():
    g = np.random.default_rng(5)
    keys = [0, 1, U64, 1 << 63, (1 << 63) - 1] + [int(v) for v in g.integers(0, 2 ** 63, 2000, dtype=np.uint64)]
    for k in keys:
        assert inv_mix64(mix64(k)) == k
        assert mix64(inv_mix64(k)) == k


def test_empty_marker_preimage():
    # the key whose record is the empty-slot marker (tests/test_gpu_grouping.py SPECIAL)
    assert mix64(0x74A6576574A65765) == U64
