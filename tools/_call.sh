set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouping.py tests/test_gpu_parity.py > gpurun_out/r04j_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04j_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so" REPS=2 bash tools/gpu_ab.sh r04j group str_card1e8 str_card1e5 > /dev/null || exit 1
grep -E "==|dedup" gpurun_out/r04j_ab.log
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" timeout -k 10 400 bash tools/gpu_pmc_kb.sh r04j_sq1 group str_card1e8 | grep -E "records|dedup_bytes|scatter_recs" 
PMC="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR" timeout -k 10 400 bash tools/gpu_pmc_kb.sh r04j_sq2 group str_card1e8 | grep -E "records|dedup_bytes|scatter_recs"
