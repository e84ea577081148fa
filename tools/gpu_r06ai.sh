set -o pipefail
# select workgroups per task (8192 / tasks instead of 2048 / tasks): parity subset on the variant, same-box A/B
cd /root/repo; mkdir -p gpurun_out; export TMPDIR=/tmp
SDP_LIBRARY=build_ab/libsdp_hb.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG:-r06ai}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG:-r06ai}_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=build_ab/libsdp_head.so hb=build_ab/libsdp_hb.so" bash tools/gpu_bench_ab.sh ${TAG:-r06ai} 3 > /dev/null || exit 1
TAG=${TAG:-r06ai} python3 - <<'PY'
import json
for leg in ('head','hb'):
    for rep in (1,2,3):
        d=json.loads(open('gpurun_out/%s_%s_%d.json'%(__import__('os').environ['TAG'],leg,rep)).read().strip().splitlines()[-1])
        print(leg, rep, d['ms_per_step'], 'select_batch', d['per_kernel'].get('sdp_select_batch',{}).get('ms_per_step'))
PY
