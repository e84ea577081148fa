"""Row-sharded describe() on 2 ranks (gloo, both on the box's GPU) against the
oracle on the whole table -- every table of tests/multirank_worker.py, then
the numeric tables again with the quantile slot-overflow fallback forced on
both ranks (sharded fallback select), then every table and the 4 M-row bench
table on ONE rank over nccl (RCCL) with the sharded paths forced
(SDP_FORCE_SHARDED=1: the stream-ordered all-reduces between select rounds,
all_to_all_single on device tensors, the owner exchanges, each checked to
have been issued).  The ranks are started by conftest.py's
session hook before this process initialises the GPU; this test waits for
them and checks their verdict.  Needs an MI355X."""

import pytest

from conftest import multirank_result

pytestmark = pytest.mark.gpu


def test_two_rank_sharded_describe():
    res = multirank_result(timeout=240)
    if res is None:
        pytest.fail('the multi-rank run was not started (pytest -m gpu on a GPU box starts it)')
    rc, log = res
    assert rc == 0, log[-6000:]
    runs = [l for l in log.splitlines() if l.startswith('MULTIRANK ')]
    assert runs == ['MULTIRANK OK failures=0'] * 3, log[-6000:]
    assert log.count('OK world=2') >= 11, log[-6000:]
    assert log.count('OK world=1') >= 11, log[-6000:]          # 10 tables + gk on the forced-sharded nccl rank
    assert '[calls] backend=nccl sharded=True' in log, log[-6000:]
