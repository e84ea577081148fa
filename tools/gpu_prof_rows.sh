#!/bin/bash
# rocprof kernel stats + gap census of the bench at a given row count.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pr}; ROWS=${2:-125000000}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_kt -o run -- python3 bench.py --rows $ROWS --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
f=$(find gpurun_out/${TAG}_kt -name '*kernel_trace.csv' | head -1)
cp $(find gpurun_out/${TAG}_kt -name '*kernel_stats.csv' | head -1) gpurun_out/${TAG}_kernel_stats.csv
ms=$(python3 -c "import json; print(json.load(open('gpurun_out/${TAG}_bench.json'))['ms_per_step'])")
python3 tools/gap_summary.py "$f" "$ms" > gpurun_out/${TAG}_gaps.txt
python3 - "$f" "$ms" > gpurun_out/${TAG}_busy.txt <<'PY'
import csv, sys, re
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
end = max(e for _, e, _ in ks); lo = end - float(sys.argv[2]) * 1e6
agg = {}
for s, e, n in ks:
    if s < lo: continue
    n = re.sub(r'\(.*', '', n).replace('void ', '')[:70]
    a = agg.setdefault(n, [0, 0.0]); a[0] += 1; a[1] += (e - s) / 1e6
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:40]:
    print('%8.2f ms %5d  %s' % (t, c, n))
PY
rm -rf gpurun_out/${TAG}_kt
head -3 gpurun_out/${TAG}_gaps.txt; head -25 gpurun_out/${TAG}_busy.txt
