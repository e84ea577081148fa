set -o pipefail
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_c_abi.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06aa_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r06aa_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_ab.sh r06aa 2 > /dev/null || exit 1
python3 - <<'PY'
import json
for leg in ('head','tree'):
    for rep in (1,2):
        d=json.loads(open('gpurun_out/r06aa_%s_%d.json'%(leg,rep)).read().strip().splitlines()[-1])
        pk=d['per_kernel']
        print(leg, rep, d['ms_per_step'], 'rowmask', pk.get('sdp_rowmask',{}).get('ms_per_step'), 'gram', pk.get('sdp_gram',{}).get('ms_per_step'))
PY
