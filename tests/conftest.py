import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'spark-df-profiling_amd')
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

MULTIRANK_LOG = os.path.join(ROOT, 'gpurun_out', 'pytest_multirank.log')
_MULTIRANK = {}


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP kernels run)')


def _gpu_selected(config):
    expr = (config.getoption('markexpr') or '').replace(' ', '')
    return 'gpu' in expr and 'notgpu' not in expr and os.path.exists('/dev/kfd')


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def pytest_sessionstart(session):
    """Start the 2-rank row-sharded check (tests/multirank_worker.py, gloo,
    both ranks on the box's one GPU) before this process touches the GPU: a
    process that has initialised HIP must not fork/exec children.  The ranks
    run beside the single-process GPU tests; test_gpu_multirank.py waits for
    them.  Three runs: every table, then the numeric tables with the quantile
    slot-overflow fallback forced on both ranks (2 gloo ranks), then every
    table and the 4 M-row bench table on ONE nccl (RCCL) rank with the sharded
    paths forced (SDP_FORCE_SHARDED=1)."""
    if not _gpu_selected(session.config):
        return
    os.makedirs(os.path.dirname(MULTIRANK_LOG), exist_ok=True)
    worker = os.path.join(ROOT, 'tests', 'multirank_worker.py')
    run = ('timeout -k 10 {t} {py} -m torch.distributed.run --nnodes 1 --nproc-per-node {np} '
           '--master-addr 127.0.0.1 --master-port {port} {w} {be} {only}')
    cmd = (run.format(t=300, py=sys.executable, np=2, port=_free_port(), w=worker, be='gloo', only='') + ' && ' +
           'SDP_DEBUG_QUANTILE=overflow ' +
           run.format(t=200, py=sys.executable, np=2, port=_free_port(), w=worker, be='gloo',
                      only='numeric,numeric_big') + ' && ' +
           # the RCCL branches on the box's one GPU: a one-rank nccl group with the
           # sharded paths forced (stream-ordered all-reduces between select
           # rounds, all_to_all_single on device tensors, the owner exchanges)
           'SDP_FORCE_SHARDED=1 SDP_REQUIRE_CALLS=allreduce_sum_,alltoallv_known,allgather,allgather_object ' +
           run.format(t=300, py=sys.executable, np=1, port=_free_port(), w=worker, be='nccl',
                      only='demo,numeric,numeric_big,categorical,categorical_big,dates,corr,legacy,sorted,gk,c3'))
    env = dict(os.environ, SDP_PLOT_WORKERS='0', HSA_ENABLE_IPC_MODE_LEGACY='0')
    log = open(MULTIRANK_LOG, 'w')
    _MULTIRANK['proc'] = subprocess.Popen(['bash', '-c', cmd], cwd=ROOT, env=env, stdout=log,
                                          stderr=subprocess.STDOUT, start_new_session=True)
    _MULTIRANK['log'] = log
    # the vectorised oracle's worker processes (C2 at 1e8 rows), likewise
    # spawned before this process initialises the GPU; 16 = the box's CPU share
    from oracle import fast
    fast.start_pool(min(16, os.cpu_count() or 1))


def multirank_result(timeout):
    """(returncode, log text) of the session's multi-rank run, or None."""
    proc = _MULTIRANK.get('proc')
    if proc is None:
        return None
    try:
        rc = proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        import signal
        os.killpg(proc.pid, signal.SIGKILL)
        rc = proc.wait()
    _MULTIRANK['log'].flush()
    with open(MULTIRANK_LOG) as fh:
        return rc, fh.read()


def pytest_sessionfinish(session, exitstatus):
    proc = _MULTIRANK.get('proc')
    if proc is not None and proc.poll() is None:
        import signal
        os.killpg(proc.pid, signal.SIGKILL)
        proc.wait()
