"""Row-sharded describe() on 2 ranks (gloo, both on the box's GPU) against the
oracle on the whole table -- every table of tests/multirank_worker.py, then
the numeric tables again with the quantile slot-overflow fallback forced on
both ranks (sharded fallback select).  The ranks are started by conftest.py's
session hook before this process initialises the GPU; this test waits for
them and checks their verdict.  Needs an MI355X."""

import pytest

from conftest import multirank_result

pytestmark = pytest.mark.gpu


def test_two_rank_sharded_describe():
    res = multirank_result(timeout=110)
    if res is None:
        pytest.fail('the multi-rank run was not started (pytest -m gpu on a GPU box starts it)')
    rc, log = res
    assert rc == 0, log[-6000:]
    runs = [l for l in log.splitlines() if l.startswith('MULTIRANK ')]
    assert runs == ['MULTIRANK OK failures=0'] * 2, log[-6000:]
    assert log.count('OK world=2') >= 10, log[-6000:]
