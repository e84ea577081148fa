#!/bin/bash
# A/B of two builds of libsdp.so on the same box: kbench stages, alternating.
# usage: tools/gpu_ab.sh TAG STAGE COL [COL...]   (A = abtest/libsdp_head.so, B = in-tree)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; ST=$2; shift 2
for c in "$@"; do
  for v in ${ABSEQ:-A B A B}; do
    if [ $v = A ]; then L=abtest/libsdp_head.so; else L=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so; fi
    echo "== $v $c" >> gpurun_out/${T}_ab.log
    SDP_LIBRARY=$L timeout -k 10 240 python -u tools/kbench.py $ST 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
  done
done
cat gpurun_out/${T}_ab.log
