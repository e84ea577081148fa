set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_grouping.py -k "distinct32" > gpurun_out/r04h_tests.log 2>&1; rc=$?
tail -12 gpurun_out/r04h_tests.log; [ $rc -eq 0 ] || exit $rc
T=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so
LIBS="tree=$T nowords=build_ab/libsdp_xNOWORDS.so noheavy=build_ab/libsdp_xNOHEAVY.so noheavycnt=build_ab/libsdp_xNOHEAVYCNT.so nostore=build_ab/libsdp_xNOSTORE.so" REPS=1 bash tools/gpu_ab.sh r04g group str_card1e8 str_card100 str_card1e5 > /dev/null || exit 1
grep -E "==|records" gpurun_out/r04g_ab.log
