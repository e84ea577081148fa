#!/bin/bash
# pass 1 with bare v_min/v_max_f64 (default) vs fmin/fmax (fminmax variant): kbench pass1b per 1e9-row column,
# then the quantile/moment GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-r03al}
for c in f64_norm f32_norm i64_uniform_2p31; do
  for rep in 1 2; do
    for lib in default fminmax; do
      if [ $lib = default ]; then unset SDP_LIBRARY; else export SDP_LIBRARY=$PWD/build_ab/libsdp_$lib.so; fi
      echo "== $lib $c" >> gpurun_out/${T}_kb.log
      timeout -k 10 240 python -u tools/kbench.py pass1b 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/${T}_kb.log || exit 1
    done
  done
done
unset SDP_LIBRARY
grep -E "==|sdp_pass1" gpurun_out/${T}_kb.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_scale_1e9.py > gpurun_out/${T}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${T}_tests.log; exit $rc
