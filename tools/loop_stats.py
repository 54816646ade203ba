"""Instruction mix of the loops of one kernel in a `hipcc -S` listing: every backward branch
(s_cbranch_* / s_branch to an earlier label) closes a loop; report its instruction counts."""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read()
kern = sys.argv[2]
m = re.search(r'^(_Z\S*' + kern + r'\S*):.*?^\s*s_endpgm', src, re.S | re.M)
lines = [l.strip() for l in m.group(0).split('\n')]
labels = {}
ins = []
for l in lines:
    if re.match(r'^\.LBB\S+:', l):
        labels[l.split(':')[0]] = len(ins)
        continue
    if not l or l.startswith(('.', ';')) or l.endswith(':'):
        continue
    ins.append(l)
for i, l in enumerate(ins):
    mm = re.match(r'^s_(cbranch_\w+|branch)\s+(\.LBB\S+)', l)
    if mm and mm.group(2) in labels and labels[mm.group(2)] <= i:
        body = [x.split()[0] for x in ins[labels[mm.group(2)]:i + 1]]
        c = Counter(body)
        print(f"loop {mm.group(2)}: {len(body)} instructions")
        print('  ' + ' '.join(f"{k}:{v}" for k, v in sorted(c.items(), key=lambda x: -x[1])[:30]))
