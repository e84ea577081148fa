set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_c_abi.py > gpurun_out/r04c_tests.log 2>&1; rc=$?
tail -40 gpurun_out/r04c_tests.log; exit $rc
