"""HBM bytes per dispatch of every sdp kernel from rocprofv3 counter CSVs.

usage: python tools/traffic_summary.py OUT.json ROWS[:WORKLOAD] DIR [DIR ...]

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced read (MI355X_MICROARCH.md, "HBM [CDNA4]"),
so traffic = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024 bytes.  Written as a
small JSON keyed by kernel name (template arguments kept, parameters dropped);
bench.py reads it for the dominant kernel's `roofline.traffic`.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]
rows, _, workload = sys.argv[2].partition(':')
rows, workload = int(rows), workload or 'c3'
vals = defaultdict(lambda: defaultdict(list))          # kernel -> counter -> per-dispatch values
for d in sys.argv[3:]:
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r['Kernel_Name'].split('(')[0].replace('void ', '').strip()
                vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
res = {}
for k, c in sorted(vals.items()):
    f, w = c.get('FETCH_SIZE', []), c.get('WRITE_SIZE', [])
    if not f or not w:
        continue
    fb = 2.0 * 1024.0 * sum(f) / len(f)
    wb = 1024.0 * sum(w) / len(w)
    res[k] = {'dispatches': max(len(f), len(w)), 'fetch_bytes': round(fb), 'write_bytes': round(wb),
              'traffic_bytes': round(fb + wb)}
with open(out, 'w') as fh:
    json.dump({'rows': rows, 'workload': workload, 'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one pass each, '
                                       'bench.py --steps 1 --warmup 0; FETCH_SIZE x2 (gfx950), KiB -> bytes',
               'kernels': res}, fh, indent=1)
print('wrote', out, len(res), 'kernels')
