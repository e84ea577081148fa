#!/bin/bash
# 2- and 3-rank row-sharded describe() vs the oracle (gloo, ranks share the GPU),
# then the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
for w in 2 3; do
  timeout -k 10 400 python -u -m torch.distributed.run --nproc-per-node $w --master-addr 127.0.0.1 --master-port 2951$w \
     tests/multirank_worker.py gloo > gpurun_out/mr_$w.log 2>&1 || { echo "world $w failed"; tail -30 gpurun_out/mr_$w.log; exit 1; }
  grep -E "OK|MISMATCH|missing" gpurun_out/mr_$w.log
done
[ "${TESTS:-1}" = 1 ] || exit 0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mr_tests.log 2>&1 || { tail -30 gpurun_out/mr_tests.log; exit 1; }
tail -2 gpurun_out/mr_tests.log
