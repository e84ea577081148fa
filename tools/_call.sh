set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_edges.py > gpurun_out/r04e_tests.log 2>&1; rc=$?
tail -30 gpurun_out/r04e_tests.log; [ $rc -eq 0 ] || exit $rc
for c in f32_norm i64_uniform_2p31; do
  for st in d32 group; do
    echo "== $st $c" >> gpurun_out/r04e_kb.log
    timeout -k 10 240 python -u tools/kbench.py $st 1000000000 2 $c 2>&1 | grep -v amdgpu.ids | tail -n +3 >> gpurun_out/r04e_kb.log || exit 1
  done
done
cat gpurun_out/r04e_kb.log
for mode in 0 1; do
  SDP_FORCE_SHARDED=$mode timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04e_125m_$mode.json 2> gpurun_out/r04e_125m_$mode.err || { tail -20 gpurun_out/r04e_125m_$mode.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r04e_125m_$mode.json').read().strip().splitlines()[-1]);print('125m forced_sharded=$mode', d['ms_per_step'], 'readbacks', d['host_readbacks_per_step'], d['roofline']['traffic_over_alg'])"
done
