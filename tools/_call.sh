set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests/test_gpu_edges.py::test_uint32_wide_fused_group tests/test_gpu_scale_1e9.py "tests/test_gpu_baseline_sizes.py::test_c4_high_cardinality_1e9" > gpurun_out/r04b_tests.log 2>&1; rc=$?
tail -15 gpurun_out/r04b_tests.log; exit $rc
