"""Idle gaps between consecutive kernels of the last describe() step in a
rocprofv3 kernel trace: python tools/gap_summary.py kernel_trace.csv [step_ms]

Prints the total busy / idle time of the final `step_ms` window and the
largest gaps keyed by the kernel that preceded them."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
step_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 600.0
ks = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)
end = max(e for _, e, _ in ks)
lo = end - step_ms * 1e6
win = [k for k in ks if k[0] >= lo]
busy, gaps, cur = 0, defaultdict(lambda: [0, 0.0]), None
for s, e, name in win:
    if cur is not None:
        g = s - cur[1]
        if g > 0:
            key = cur[2].split('(')[0][:60]
            gaps[key][0] += 1
            gaps[key][1] += g / 1e6
    if cur is None or e > cur[1]:
        busy += e - max(s, cur[1] if cur else s)
        cur = (s, e, name)
span = (win[-1][1] - win[0][0]) / 1e6
print('window %.1f ms: %d kernels, busy %.1f ms, idle %.1f ms' % (span, len(win), busy / 1e6, span - busy / 1e6))
for k, (c, t) in sorted(gaps.items(), key=lambda kv: -kv[1][1])[:25]:
    print('  %8.2f ms idle after %5d x %s' % (t, c, k))
