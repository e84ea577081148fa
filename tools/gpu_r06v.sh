set -o pipefail
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_owner_order.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r06v}_tests.log 2>&1
rc=$?; tail -5 gpurun_out/${TAG:-r06v}_tests.log; cp gpurun_out/pytest_multirank.log gpurun_out/${TAG:-r06v}_multirank.log 2>/dev/null
[ $rc -eq 0 ] || exit $rc
NOPROF=1 bash tools/gpu_rank_share.sh ${TAG:-r06v}
