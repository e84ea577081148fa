set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ingest.py tests/test_gpu_edges.py > gpurun_out/r04d_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r04d_tests.log; exit $rc
