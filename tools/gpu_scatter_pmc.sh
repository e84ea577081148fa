#!/bin/bash
# Row-scatter counters per dispatch under several allocator states
# (tools/scatter_alloc_probe.py): translation (UTCL1) and DRAM write-stall
# counters in separate passes, joined with each dispatch's duration.
# usage: tools/gpu_scatter_pmc.sh TAG
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${1:-spmc}
i=0
for ctrs in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum" \
            "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_DRAM_sum"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --kernel-trace --output-format csv --pmc $ctrs --kernel-include-regex 'part_scatter_rows' \
      -d gpurun_out/${T}_p$i -o run -- python3 tools/scatter_alloc_probe.py > gpurun_out/${T}_p$i.log 2>&1 \
      || { tail -5 gpurun_out/${T}_p$i.log; exit 1; }
done
python3 - gpurun_out/${T} > gpurun_out/${T}_scatter_pmc.txt <<'PY'
import csv, glob, sys, collections
base = sys.argv[1]
for p in (1, 2):
    rows = collections.defaultdict(dict)
    for f in glob.glob('%s_p%d/**/*counter_collection.csv' % (base, p), recursive=True):
        for r in csv.DictReader(open(f)):
            d = r.get('Dispatch_Id') or r.get('Correlation_Id')
            rows[d][r['Counter_Name']] = float(r['Counter_Value'])
            if 'End_Timestamp' in r and r.get('Start_Timestamp'):
                rows[d]['ms'] = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6
    for d in sorted(rows, key=lambda x: int(x)):
        print('pass', p, 'dispatch', d, '  '.join('%s %.4g' % kv for kv in sorted(rows[d].items())))
PY
cat gpurun_out/${T}_scatter_pmc.txt
grep -v amdgpu.ids gpurun_out/${T}_p1.log | tail -12
rm -rf gpurun_out/${T}_p1 gpurun_out/${T}_p2
