#!/bin/bash
# kbench STAGE on 1e9-row columns: default library vs build_ab/libsdp_$V.so, alternating.
# usage: tools/gpu_lib_kb.sh TAG V STAGE COL [COL...]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=$1; V=$2; ST=$3; shift 3
for c in "$@"; do
  for lib in default $V default $V; do
    if [ $lib = default ]; then unset SDP_LIBRARY; else export SDP_LIBRARY=$PWD/build_ab/libsdp_$lib.so; fi
    echo "== $lib $c" >> gpurun_out/${T}_kb.log
    timeout -k 10 240 python -u tools/kbench.py $ST 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_kb.log || exit 1
  done
done
grep -E "==|part_" gpurun_out/${T}_kb.log
