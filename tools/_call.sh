set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_c_abi.py tests/test_gpu_configs.py > gpurun_out/r04t_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04t_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so" REPS=3 bash tools/gpu_ab.sh r04t gram f64_norm > /dev/null || exit 1
grep -E "==|gram" gpurun_out/r04t_ab.log
