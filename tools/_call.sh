set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_c_abi.py tests/test_gpu_multirank.py tests/test_gpu_configs.py > gpurun_out/r04za_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04za_tests.log; exit $rc
