#!/bin/bash
# pass-1 32-bit window keys: kbench pass1b per 1e9-row column, default (key32, slots widened after the sweep) vs
# nok32 (64-bit keys) vs inline (widened in the store branch) vs skipw (never widened: the compare-only cost; wrong quantiles).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r03ak}
for c in f32_norm f32_uniform date; do
  for rep in 1 2; do
    for lib in default nok32 inline skipw; do
      if [ $lib = default ]; then unset SDP_LIBRARY; else export SDP_LIBRARY=$PWD/build_ab/libsdp_$lib.so; fi
      echo "== $lib $c" >> gpurun_out/${T}_kb.log
      timeout -k 10 240 python -u tools/kbench.py pass1b 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_kb.log || exit 1
    done
  done
done
grep -E "==|pass1_batch|sdp_pass1" gpurun_out/${T}_kb.log
