#!/bin/bash
# SQ counters of the sdp kernels of one kbench stage on one 1e9-row column,
# under each environment setting (same box): two passes (timing-shape
# counters, instruction counts), one rocprofv3 run each.
# usage: tools/gpu_pmc_env.sh TAG STAGE COL "SET_A SET_B"
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; STAGE=$2; COL=$3; SETS=$4
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS"
for v in $SETS; do
  for pi in 1 2; do
    [ $pi = 1 ] && P=$P1 || P=$P2
    d=gpurun_out/${T}_${v//[=,]/_}_$pi
    env ${v//,/ } timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $P \
      --kernel-include-regex 'sdp::' -d $d -o run -- python3 tools/kbench.py $STAGE 1000000000 1 $COL \
      > $d.log 2>&1 || { tail -5 $d.log; exit 1; }
    echo "== $v pass $pi" >> gpurun_out/${T}_pmc.txt
    python3 tools/pmc_table.py $d >> gpurun_out/${T}_pmc.txt
    rm -rf $d
  done
done
cat gpurun_out/${T}_pmc.txt
