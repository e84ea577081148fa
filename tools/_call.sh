set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_bench.sh r04i || exit 1
bash tools/gpu_traffic.sh r04i || exit 1
