#!/bin/bash
# SQ counters of the sdp kernels of one kbench stage on one 1e9-row column.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${1:-pk}; STAGE=${2:-group}; COL=${3:-str_card1e8}
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv \
  --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT} \
  --kernel-include-regex 'sdp::' -d gpurun_out/${T}_pmc -o run -- python3 tools/kbench.py $STAGE 1000000000 1 $COL \
  > gpurun_out/${T}_pmc.log 2>&1 || { tail -5 gpurun_out/${T}_pmc.log; exit 1; }
python3 - gpurun_out/${T}_pmc > gpurun_out/${T}_pmc.txt <<'PY'
import csv, glob, sys, collections
v = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]
        v[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in v.items():
    if 'SQ_WAIT_ANY' not in c:
        print('%-60s %s' % (k, '  '.join('%s %.4g' % kv for kv in sorted(c.items()))))
        continue
    wc = c['SQ_WAVE_CYCLES'] or 1
    print('%-60s wave_cyc %.3g  wait_any %.2f  wait_inst %.2f  active %.2f  valu %.2f  lds %.2f  bankconf/lds %.2f' % (
        k, wc, c['SQ_WAIT_ANY'] / wc, c['SQ_WAIT_INST_ANY'] / wc, c['SQ_ACTIVE_INST_ANY'] / wc,
        c['SQ_ACTIVE_INST_VALU'] / wc, c['SQ_ACTIVE_INST_LDS'] / wc,
        c['SQ_LDS_BANK_CONFLICT'] / max(1, c['SQ_ACTIVE_INST_LDS'])))
PY
rm -rf gpurun_out/${T}_pmc
cat gpurun_out/${T}_pmc.txt
