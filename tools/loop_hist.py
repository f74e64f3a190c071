"""Opcode histogram of the innermost (feature) loop of a kernel in an asm listing.
Usage: python tools/loop_hist.py build/sbz_lik.s <mangled-kernel-substring>"""
import re
import sys
from collections import Counter

asm, name = sys.argv[1], sys.argv[2]
L = open(asm).read().split('\n')
s = next(i for i, l in enumerate(L) if l.startswith('_ZN') and name in l and l.split(';')[0].rstrip().endswith(':'))
e = next(i for i in range(s, len(L)) if 's_endpgm' in L[i])
K = L[s:e + 1]
hdr = [i for i, l in enumerate(K) if 'Loop Header' in l and 'Depth=2' in l]
if not hdr:
    hdr = [i for i, l in enumerate(K) if 'Loop Header' in l]
h = hdr[0]
j = h
while not K[j].startswith('.LBB'):
    j -= 1
bb = K[j].split(':')[0][1:]  # e.g. LBB38_13 -> header name BB38_13
key = 'Header=' + bb[1:]
# lines of every basic block that belongs to this loop (label comment names the header)
body, inside = [], False
for i, l in enumerate(K):
    if l.startswith('.LBB'):
        inside = (i == j) or (key in l) or (key in K[i + 1] if i + 1 < len(K) else False)
    if inside:
        body.append(l)
lab, h, end = bb, j, j + len(body)
ops, cats = Counter(), Counter()
for l in body:
    t = l.strip().split()
    if not t or t[0].startswith(('.', ';')):
        continue
    op = t[0]
    cat = ('valu' if op.startswith('v_') else 'lds' if op.startswith('ds_') else
           'vmem' if op.startswith(('global_', 'buffer_')) else 'wait' if op.startswith('s_waitcnt')
           else 'salu' if op.startswith('s_') else 'other')
    cats[cat] += 1
    if cat == 'valu':
        ops[op] += 1
print(f"loop {lab} lines {h}..{end}: {dict(cats)}")
for k, v in ops.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 30):
    print(f"{v:5d} {k}")
