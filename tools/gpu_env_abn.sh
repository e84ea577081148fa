#!/bin/bash
# A/B/C.. of one environment switch on the same build: kbench STAGE on 1e9-row columns,
# two rounds over VALUES.  usage: tools/gpu_env_abn.sh TAG STAGE VAR "V1 V2 .." COL [COL...]
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=$1; ST=$2; VAR=$3; VALS=$4; shift 4
for c in "$@"; do
  for rep in 1 2; do
    for v in $VALS; do
      echo "== $VAR=$v $c" >> gpurun_out/${T}_ab.log
      env $VAR=$v timeout -k 10 240 python -u tools/kbench.py $ST 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_ab.log || exit 1
    done
  done
done
grep -E "==|dedup" gpurun_out/${T}_ab.log
