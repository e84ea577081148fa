"""Static instruction mix of a kernel's hottest loop in a gfx950 .s file:
python tools/isa_loop.py FILE.s SYMBOL_SUBSTRING [ELEMS_PER_ITER [LOOP_INDEX]]
Counts VALU / SALU / memory instructions between the loop header with the
most instructions and its back edge, excluding blocks whose label shows they
are rarely taken (none excluded; prints the per-block counts instead)."""
import re
import sys
from collections import Counter

path, sym = sys.argv[1], sys.argv[2]
per = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0
lines = open(path).read().split('\n')
start = next(i for i, l in enumerate(lines) if re.match(r'^_Z\S*%s\S*:' % re.escape(sym), l))
end = next(i for i in range(start + 1, len(lines)) if lines[i].startswith('.Lfunc_end'))
body = lines[start:end]
# loop headers: labels followed by '; =>This Inner Loop Header' comment
best = None
pick = int(sys.argv[4]) if len(sys.argv) > 4 else None
loops = []
for i, l in enumerate(body):
    m = re.match(r'^(\.LBB\d+_\d+):.*Loop Header', l)
    if not m:
        continue
    lab = m.group(1)
    back = max((k for k in range(i, len(body)) if re.search(r's_cbranch\w*\s+%s$|s_branch\s+%s$' % (lab, lab), body[k])),
               default=None)
    if back is None:
        continue
    seg = [x.strip() for x in body[i:back + 1]]
    ins = [x for x in seg if x and not x.startswith(';') and not x.startswith('.')]
    loops.append((lab, ins, seg))
    if best is None or len(ins) > len(best[1]):
        best = (lab, ins, seg)
print('loops:', ', '.join('%d:%s(%d)' % (k, a, len(b)) for k, (a, b, _) in enumerate(loops)))
lab, ins, seg = loops[pick] if pick is not None else best
ops = Counter(x.split()[0] for x in ins)
v = sum(c for o, c in ops.items() if o.startswith('v_'))
s_ = sum(c for o, c in ops.items() if o.startswith('s_'))
mem = sum(c for o, c in ops.items() if o.startswith(('global_', 'flat_', 'buffer_', 'ds_')))
print('%s loop %s: %d instr, VALU %d, SALU %d, mem %d (per elem: %.1f / %.1f)' % (sym, lab, len(ins), v, s_, mem, v / per, s_ / per))
for o, c in ops.most_common(40):
    print('  %5d %s' % (c, o))
