#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_round3.sh r03af || exit 1
timeout -k 10 400 python -u tools/c5_profile.py > gpurun_out/r03af_c5.log 2>&1 || { tail -20 gpurun_out/r03af_c5.log; exit 1; }
head -12 gpurun_out/r03af_c5.log
timeout -k 10 300 python -u bench.py --workload c5 --rows 10000000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03af_c5_bench.json 2> gpurun_out/r03af_c5_bench.err || { tail -20 gpurun_out/r03af_c5_bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/r03af_c5_bench.json').read().strip().splitlines()[-1]);print('c5 bench with plots', d['ms_per_step'], d['roofline'].get('frac'))"
