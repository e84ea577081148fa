#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_multirank.py tests/test_gpu_ragged.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
bash tools/gpu_c5prof.sh ${TAG}
