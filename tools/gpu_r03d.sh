#!/bin/bash
# dedup MLP A/B + 1.25e8-row bench, single-rank vs forced-sharded (one-rank RCCL)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03d}
bash tools/gpu_dedup_mlp.sh ${TAG}_mlp || exit 1
timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_125m.json 2> gpurun_out/${TAG}_125m.err || { tail -20 gpurun_out/${TAG}_125m.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_125m.json'));print('single', d['ms_per_step'])"
SDP_FORCE_SHARDED=1 timeout -k 10 300 python -u bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_125m_sharded.json 2> gpurun_out/${TAG}_125m_sharded.err || { tail -20 gpurun_out/${TAG}_125m_sharded.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_125m_sharded.json'));print('forced-sharded', d['ms_per_step'])"
