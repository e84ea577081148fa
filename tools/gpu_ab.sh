#!/bin/bash
# Same-box A/B of builds of libsdp.so: tools/kbench.py STAGE on 1e9-row columns,
# the builds alternated per repetition.
# usage: tools/gpu_ab.sh TAG STAGE COL [COL...]
#   LIBS="name=path ..." (default: "head=abtest/libsdp_head.so tree=<in-tree>"), REPS (default 2), ROWS (default 1e9)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; ST=$2; shift 2
TREE=spark-df-profiling_amd/spark_df_profiling/lib/libsdp.so
LIBS=${LIBS:-"head=abtest/libsdp_head.so tree=$TREE"}
for c in "$@"; do
  for rep in $(seq ${REPS:-2}); do
    for nl in $LIBS; do
      name=${nl%%=*}; L=${nl#*=}
      echo "== $name $c rep $rep" >> gpurun_out/${T}_ab.log
      SDP_LIBRARY=$L timeout -k 10 240 python -u tools/kbench.py $ST ${ROWS:-1000000000} 2 $c 2>&1 \
          | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${T}_ab.log
