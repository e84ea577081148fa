#!/bin/bash
# RCCL same-GPU probe, then per-column grouping timings of the byte columns
# (partition path vs global table) at 1e9 rows.  Logs under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 tools/rccl_probe.py > gpurun_out/rccl_probe.log 2>&1
echo "rccl probe rc=$?"
tail -5 gpurun_out/rccl_probe.log
for c in str_card1e5 str_card100; do
  timeout -k 10 240 python -u tools/kbench.py group 1000000000 2 $c > gpurun_out/kb_group_$c.log 2>&1 || exit 1
  KB_CAP=$((1<<19)) timeout -k 10 240 python -u tools/kbench.py table 1000000000 2 $c > gpurun_out/kb_table_$c.log 2>&1 || exit 1
done
tail -n 12 gpurun_out/kb_*.log
bash tools/gpu_pmc_kb.sh pk100 group str_card100
bash tools/gpu_pmc_kb.sh pk1e5 group str_card1e5
