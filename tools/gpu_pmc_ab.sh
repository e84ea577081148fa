#!/bin/bash
# SQ counters of one kbench stage on one 1e9-row column, for each library of
# LIBS (name=path ...), two counter passes each (issue shape; instruction counts).
# usage: tools/gpu_pmc_ab.sh TAG STAGE COL
#   ENVS="A,B" instead: one run per environment setting of the tree library
#   (e.g. ENVS="SDP_L2_BLOCKS=0,SDP_L2_BLOCKS=1")
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; ST=$2; C=$3
LIBS=${LIBS:-"head=build_ab/libsdp_head.so tree=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so"}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH"
if [ -n "$ENVS" ]; then
  LIBS=""
  for e in ${ENVS//,/ }; do LIBS="$LIBS ${e//=/_}=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so"; done
fi
for nl in $LIBS; do
  name=${nl%%=*}; L=${nl#*=}
  EV=""; [ -n "$ENVS" ] && EV=$(echo $name | sed 's/_\([0-9]*\)$/=\1/')
  k=0
  for P in "$P1" "$P2"; do
    k=$((k+1))
    env $EV SDP_LIBRARY=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $P \
      --kernel-include-regex 'sdp::' -d gpurun_out/${T}_${name}_p$k -o run -- python3 tools/kbench.py $ST 1000000000 1 $C \
      > gpurun_out/${T}_${name}_p$k.log 2>&1 || { tail -5 gpurun_out/${T}_${name}_p$k.log; exit 1; }
    echo "== $name pass $k $ST $C" >> gpurun_out/${T}_pmc.txt
    python3 tools/pmc_table.py gpurun_out/${T}_${name}_p$k >> gpurun_out/${T}_pmc.txt
    rm -rf gpurun_out/${T}_${name}_p$k
  done
done
cat gpurun_out/${T}_pmc.txt
