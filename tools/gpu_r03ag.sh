#!/bin/bash
# multi-rank bench harness rehearsal: 2 and 4 gloo ranks sharing the box's GPU (the driver's N>1 launch line)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for N in 2 4; do
  SDP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29540 + N)) bench.py --gpus $N --rows 40000000 --steps 2 --warmup 1 > gpurun_out/r03ag_n$N.json 2> gpurun_out/r03ag_n$N.err || { tail -30 gpurun_out/r03ag_n$N.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/r03ag_n$N.json').read().strip().splitlines()[-1]);print('N=$N', d['n_gpus'], d['ms_per_step'], d['value'], d['config']['parallelism'])"
done
