#!/bin/bash
# Round-2 profile set: C3 bench line, rocprof kernel stats, PMC traffic; the
# same for C5.  Everything under gpurun_out/<tag>_*.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-r02}
timeout -k 10 400 python3 -u bench.py --steps 10 --warmup 3 > gpurun_out/${T}_c3_bench.json 2> gpurun_out/${T}_c3_bench.err &&
echo "c3 bench ok" &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c3_kt -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_c3_prof.json 2> gpurun_out/${T}_c3_prof.err &&
cp $(find gpurun_out/${T}_c3_kt -name '*kernel_stats.csv' | head -1) gpurun_out/${T}_c3_kernel_stats.csv && rm -rf gpurun_out/${T}_c3_kt &&
echo "c3 rocprof ok" &&
bash tools/gpu_traffic.sh ${T}_c3 1000000000 &&
timeout -k 10 300 python3 -u bench.py --workload c5 --steps 3 --warmup 1 > gpurun_out/${T}_c5_bench.json 2> gpurun_out/${T}_c5_bench.err &&
echo "c5 bench ok" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_c5_kt -o run -- \
    python3 bench.py --workload c5 --steps 2 --warmup 1 --no-plots > gpurun_out/${T}_c5_prof.json 2> gpurun_out/${T}_c5_prof.err &&
cp $(find gpurun_out/${T}_c5_kt -name '*kernel_stats.csv' | head -1) gpurun_out/${T}_c5_kernel_stats.csv && rm -rf gpurun_out/${T}_c5_kt &&
echo "c5 rocprof ok" &&
BENCH_ARGS="--workload c5 --no-plots" bash tools/gpu_traffic.sh ${T}_c5 10000000
