"""Instruction mix of the innermost loop of a kernel in a hipcc -S file (every basic block
annotated with the innermost loop header, so rarely taken paths inside the loop count too).
usage: python tools/loop_mix.py file.s kernel_substring"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
name = [m for m in re.findall(r'^(_Z\S*?):', s, re.M) if sys.argv[2] in m][0]
body = s[s.index(name + ':'):]
body = body[:body.index('.Lfunc_end')]
lines = body.split('\n')
depth = max(int(d) for d in re.findall(r'Depth=(\d+)', body))
hdr = re.search(r'Header=(BB\d+_\d+) Depth=%d' % depth, body).group(1)
c, blocks, inloop = Counter(), 0, False
for l in lines:
    if re.match(r'^(\.LBB|; %bb)', l):
        inloop = (('Header=%s' % hdr) in l) or l.startswith('.L' + hdr + ':')
        blocks += inloop
        continue
    t = l.strip().split()
    if not inloop or not t or t[0].startswith(('.', ';')):
        continue
    op = re.sub(r'_e(32|64)$|_sdwa$|_dpp$', '', t[0])
    cls = ('VALU' if op.startswith('v_') else 'LDS' if op.startswith('ds_') else
           'VMEM' if op.startswith(('global_', 'buffer_')) else
           'other' if op.startswith(('s_waitcnt', 's_cbranch', 's_branch', 's_nop')) else 'SALU')
    c[cls] += 1
    c[op] += 1
print(f'{name[:60]} innermost loop {hdr} (depth {depth}), {blocks} blocks')
print('  '.join(f'{k} {c[k]}' for k in ('VALU', 'SALU', 'LDS', 'VMEM', 'other')))
print(', '.join(f'{k} {v}' for k, v in c.most_common(45) if k not in ('VALU', 'SALU', 'LDS', 'VMEM', 'other')))
