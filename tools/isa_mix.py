"""Per-basic-block instruction mix of one kernel in a hipcc -S listing (profiling aid).
usage: python tools/isa_mix.py listing.s kernel_symbol_prefix [min_mfma]"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
k = sys.argv[2]
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 1
i = s.index('\n' + k) + 1
body = s[i:s.index('.Lfunc_end', i)]
blocks, cur, name = [], [], 'entry'
for l in body.split('\n'):
    l = l.split(';')[0].strip()
    if not l:
        continue
    m = re.match(r'^([.\w]+):', l)
    if m:
        blocks.append((name, cur))
        name, cur = m.group(1), []
        continue
    if l.startswith('.'):
        continue
    cur.append(l)
blocks.append((name, cur))
for name, b in blocks:
    c = Counter(l.split()[0] for l in b)
    nm = sum(v for op, v in c.items() if 'mfma' in op)
    br = [l for l in b if 'branch' in l]
    if nm >= lo:
        valu = sum(v for op, v in c.items() if op.startswith('v_') and 'mfma' not in op)
        print(f"{name}: {len(b)} instr, mfma {nm}, valu {valu}, branches {br}")
        print('   ', sorted(c.items(), key=lambda x: -x[1])[:28])
