set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_c_abi.py > gpurun_out/r04l_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so" REPS=2 bash tools/gpu_ab.sh r04l group f64_norm i64_zipf str_card1e8 str_card1e5 > /dev/null || exit 1
grep -E "==|dedup" gpurun_out/r04l_ab.log
