#!/bin/bash
# PMC passes (one counter set per pass) on one engine stage of a 1e9-row C3
# column: kernel counters + HBM bytes.  Usage (via gpurun):
#   COLS="f64_norm str_card1e8" WHAT=group bash tools/gpu_pmc_group.sh TAG
set -o pipefail
TAG=${1:-pmc}
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_$TAG
export TMPDIR=/tmp
WHAT=${WHAT:-group}
for c in ${COLS:-f64_norm}; do
  i=0
  for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
             "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc $set -d gpurun_out/pmc_$TAG/${c}_p$i -o run -- python3 tools/kbench.py $WHAT 1000000000 2 $c > gpurun_out/pmc_$TAG/${c}_p$i.log 2>&1 || { echo "pass $i failed for $c"; tail -5 gpurun_out/pmc_$TAG/${c}_p$i.log; exit 1; }
    echo "pmc $c pass $i ok"
  done
  python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_$c.csv gpurun_out/pmc_$TAG/${c}_p1 gpurun_out/pmc_$TAG/${c}_p2 gpurun_out/pmc_$TAG/${c}_p3 gpurun_out/pmc_$TAG/${c}_p4
done
rm -rf gpurun_out/pmc_$TAG
