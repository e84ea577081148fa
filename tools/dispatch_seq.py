"""Per-dispatch durations (in launch order) of the kernels whose names contain
a pattern, from a rocprofv3 kernel_trace.csv: which call of a step is slow.
    python tools/dispatch_seq.py KERNEL_TRACE_CSV PATTERN [PATTERN ...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
pats = sys.argv[2:]
for p in pats:
    seq = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e6 for r in rows if p in r['Kernel_Name']]
    print('%s: %d dispatches' % (p, len(seq)))
    print('  ' + ' '.join('%.2f' % x for x in seq))
