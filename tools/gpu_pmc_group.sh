#!/bin/bash
# GPU parity tests, then PMC passes on the grouping kernels (one counter set per pass).
set -e
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
echo "tests ok"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv --pmc $set -d gpurun_out/pmc/p$i -o run -- python3 tools/kbench.py group 1000000000 2 f64_norm > gpurun_out/pmc/p$i.log 2>&1
  echo "pmc pass $i ok"
done
python3 tools/pmc_summary.py gpurun_out/pmc_group_summary.csv gpurun_out/pmc/p1 gpurun_out/pmc/p2 gpurun_out/pmc/p3 gpurun_out/pmc/p4
cp gpurun_out/pmc/*.log gpurun_out/ && rm -rf gpurun_out/pmc
