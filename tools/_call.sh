set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
# tree = HEAD + cross-chunk prefetch in the record scatter (sdp_part.hip only; the
# engine and the record layout are HEAD's, so the HEAD library is a valid baseline)
LIBS="head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so" REPS=4 bash tools/gpu_ab.sh r04zc group f64_norm f64_uniform > /dev/null || exit 1
grep -E "==|u64/scatter" gpurun_out/r04zc_ab.log
