"""Aggregate rocprofv3 counter_collection CSVs: per kernel, per counter -> mean per dispatch.

usage: python tools/pmc_summary.py OUT.csv DIR [DIR ...]
Also reads kernel_trace CSVs for mean duration.  Raw dirs can be deleted after.
"""
import csv, glob, os, sys
from collections import defaultdict

out = sys.argv[1]
acc = defaultdict(lambda: defaultdict(float))     # (kernel) -> counter -> sum over dispatches
disp = defaultdict(lambda: defaultdict(set))       # kernel -> counter -> dispatch ids
dur = defaultdict(list)
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r['Kernel_Name'][:90]
                c = r['Counter_Name']
                acc[k][c] += float(r['Counter_Value'])
                disp[k][c].add(r['Dispatch_Id'])
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                dur[r['Kernel_Name'][:90]].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3)
counters = sorted({c for k in acc for c in acc[k]})
with open(out, 'w', newline='') as fh:
    w = csv.writer(fh)
    w.writerow(['kernel', 'dispatches', 'mean_us'] + counters)
    for k in sorted(acc):
        n = max(len(v) for v in disp[k].values())
        ds = dur.get(k, [])
        w.writerow([k, n, '%.1f' % (sum(ds) / len(ds)) if ds else ''] +
                   ['%.4g' % (acc[k][c] / max(len(disp[k][c]), 1)) if c in acc[k] else '' for c in counters])
print('wrote', out, len(acc), 'kernels')
