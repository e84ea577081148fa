"""bench.py's --gpus launcher (CPU): N rank children when no launcher set
WORLD_SIZE, and a rank whose world differs from --gpus exits non-zero."""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launch_cmd_spawns_ranks():
    cmd = bench.launch_cmd(['--gpus', '4', '--steps', '2'], 4, {})
    assert cmd[1:3] == ['-m', 'torch.distributed.run']
    assert cmd[cmd.index('--nproc-per-node') + 1] == '4'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert int(cmd[cmd.index('--master-port') + 1]) > 0
    assert cmd[-4:] == [os.path.abspath(bench.__file__), '--gpus', '4', '--steps', '2'][-4:]
    assert os.path.abspath(bench.__file__) in cmd


def test_launch_cmd_none_under_launcher_or_one_gpu():
    assert bench.launch_cmd(['--gpus', '8'], 8, {'WORLD_SIZE': '8'}) is None
    assert bench.launch_cmd([], 1, {}) is None


def test_check_world():
    bench.check_world(2, 2, 2)
    bench.check_world(1, 1, 1)
    with pytest.raises(SystemExit):
        bench.check_world(8, 1, 1)          # the silent one-GPU run of an 8-GPU point
    with pytest.raises(SystemExit):
        bench.check_world(2, 2, 1)          # a rank missing from the collective


def test_run_ranks_reprints_rank0_line_and_rc(capsys):
    ok = [sys.executable, '-c', 'print("log line"); print(\'{"value": 1, "n_gpus": 2}\')']
    assert bench.run_ranks(ok) == 0
    out = capsys.readouterr()
    assert out.out.strip() == '{"value": 1, "n_gpus": 2}'
    assert 'log line' in out.err
    bad = [sys.executable, '-c', 'import sys; sys.exit(3)']
    assert bench.run_ranks(bad) == 3
    silent = [sys.executable, '-c', 'pass']
    assert bench.run_ranks(silent) == 1


@pytest.mark.parametrize('label', ['sdp_part_rows[f64/scatter]', 'sdp_part_rows[i64/scatter]',
                                   'sdp_part_rows_records[bytes/records]', 'sdp_part_dedup_blocks[u64]',
                                   'sdp_part_l2_blocks[u64/l2blocks]', 'sdp_pass1_batch[f64/batch]'])
def test_committed_traffic_summary_covers_dominant_kernels(label):
    """roofline.traffic comes from the committed PMC summary: each kernel that
    has been the C3 bench's dominant one must map to its rocprof name there."""
    path = bench.TRAFFIC_SUMMARY['c3']
    traffic, src = bench.pmc_traffic(label, path, 1_000_000_000, 'c3')
    assert src == path and traffic > 0
