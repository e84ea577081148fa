#!/bin/bash
# A/B of one environment switch on the same build: kbench STAGE on 1e9-row columns,
# alternating VAR=A / VAR=B.  usage: tools/gpu_env_ab.sh TAG STAGE VAR A B COL [COL...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; ST=$2; VAR=$3; A=$4; B=$5; shift 5
for c in "$@"; do
  for v in $A $B $A $B; do
    echo "== $VAR=$v $c" >> gpurun_out/${T}_ab.log
    env $VAR=$v timeout -k 10 240 python -u tools/kbench.py $ST 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
  done
done
cat gpurun_out/${T}_ab.log
