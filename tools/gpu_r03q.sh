#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r03q}
timeout -k 10 300 python -u tools/step_profile.py 125000000 1 0 > gpurun_out/${TAG}_stepprof_1.log 2>&1 || { tail -20 gpurun_out/${TAG}_stepprof_1.log; exit 1; }
grep "step ms" gpurun_out/${TAG}_stepprof_1.log
SDP_FORCE_SHARDED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --rows 125000000 --steps 5 --warmup 2 --no-cpu-baseline --no-plots > gpurun_out/${TAG}_shd5.json 2> gpurun_out/${TAG}_shd5.err || { tail -20 gpurun_out/${TAG}_shd5.err; exit 1; }
f=$(find gpurun_out/${TAG}_kt -name '*kernel_trace.csv' | head -1); gzip -c "$f" > gpurun_out/${TAG}_shd5_kernel_trace.csv.gz; rm -rf gpurun_out/${TAG}_kt
bash tools/gpu_c5prof.sh ${TAG}
