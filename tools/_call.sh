set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_c_abi.py > gpurun_out/r04k_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04k_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so bst=build_ab/libsdp_bst.so" REPS=2 bash tools/gpu_ab.sh r04k group str_card1e8 str_card1e5 > /dev/null || exit 1
grep -E "==|records|scatter_rows_bytes|count_rows_bytes|group str" gpurun_out/r04k_ab.log
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" timeout -k 10 400 bash tools/gpu_pmc_kb.sh r04k_sq1 group str_card1e8 | grep -E "records|dedup_bytes|scatter_recs"
