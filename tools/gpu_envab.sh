#!/bin/bash
# Same-box A/B of environment settings of the in-tree library: tools/kbench.py
# STAGE on 1e9-row columns, the settings alternated per repetition.
# usage: tools/gpu_envab.sh TAG STAGE "SET_A SET_B ..." COL [COL...]
#   a setting is VAR=VAL[,VAR=VAL...]; REPS (default 2), ROWS (default 1e9)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; ST=$2; SETS=$3; shift 3
for c in "$@"; do
  for rep in $(seq ${REPS:-2}); do
    for v in $SETS; do
      echo "== $v $c rep $rep" >> gpurun_out/${T}_ab.log
      env ${v//,/ } timeout -k 10 240 python -u tools/kbench.py $ST ${ROWS:-1000000000} 2 $c 2>&1 \
          | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
    done
  done
done
cat gpurun_out/${T}_ab.log
