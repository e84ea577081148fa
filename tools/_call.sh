set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_parity.py tests/test_gpu_grouping.py tests/test_gpu_configs.py > gpurun_out/r04rd_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04rd_tests.log; [ $rc -eq 0 ] || exit $rc
SDP_READBACK_SITES=1 SDP_FORCE_SHARDED=1 timeout -k 10 300 python -u bench.py --rows 125000000 --steps 3 --warmup 2 --no-cpu-baseline > gpurun_out/r04rd_shd.json 2> gpurun_out/r04rd_shd.err || exit 1
grep "readback site" gpurun_out/r04rd_shd.err
python3 -c "import json;d=json.loads(open('gpurun_out/r04rd_shd.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['host_readbacks_per_step'])"
