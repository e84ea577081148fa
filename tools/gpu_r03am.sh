#!/bin/bash
# byte records kernel: two-stage (default, 4 waves/SIMD) vs three-stage pipeline (brec3: 3 waves/SIMD, 768-block grid; brec3g: 1024 blocks):
# kbench group on 1e9-row string columns, then the byte-path GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r03am}
for c in str_card1e8 str_card100; do
  for rep in 1 2; do
    for lib in default brec3 brec3g; do
      if [ $lib = default ]; then unset SDP_LIBRARY; else export SDP_LIBRARY=$PWD/build_ab/libsdp_$lib.so; fi
      echo "== $lib $c" >> gpurun_out/${T}_kb.log
      timeout -k 10 240 python -u tools/kbench.py group 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_kb.log || exit 1
    done
  done
done
unset SDP_LIBRARY
grep -E "==|records|rep 1" gpurun_out/${T}_kb.log
SDP_LIBRARY=$PWD/build_ab/libsdp_brec3.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_grouping.py tests/test_gpu_parity.py tests/test_gpu_baseline_sizes.py > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.log; exit $rc
