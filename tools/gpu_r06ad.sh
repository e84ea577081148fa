set -o pipefail
# batched radix select change: GPU suite, then same-box bench A/B
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
[ -n "$NOTEST" ] || timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${TAG:-r06ad}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG:-r06ad}_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_ab.sh ${TAG:-r06ad} ${REPS:-2} > /dev/null || exit 1
TAG=${TAG:-r06ad} REPS=${REPS:-2} python3 - <<'PY'
import json, os
T = os.environ['TAG']
for leg in ('head','tree'):
    for rep in range(1, int(os.environ.get("REPS", "2")) + 1):
        d=json.loads(open('gpurun_out/%s_%s_%d.json'%(T,leg,rep)).read().strip().splitlines()[-1])
        pk=d['per_kernel']
        print(leg, rep, d['ms_per_step'], 'select_batch', pk.get('sdp_select_batch',{}).get('ms_per_step'))
PY
