#!/bin/bash
# SQ counters of the grouping kernels of several 1e9-row columns (tools/gpu_pmc_kb.sh per column).
set -o pipefail
cd "$(dirname "$0")/.."
T=${1:-pp}; shift
for c in "$@"; do
  bash tools/gpu_pmc_kb.sh ${T}_$c group $c || exit 1
done
