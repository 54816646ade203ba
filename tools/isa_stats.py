"""Per-kernel ISA statistics from a `hipcc --cuda-device-only -S` listing: instruction mix,
LDS reads and lgkmcnt waits (how well LDS latency is pipelined), VGPRs, scratch."""
import re
import sys
from collections import Counter

src = open(sys.argv[1]).read()
pat = re.compile(r'^(_Z\S+):\s*;\s*@\S+\n(.*?)^\s*s_endpgm', re.S | re.M)
for m in pat.finditer(src):
    name = re.search(r'(k_[a-z0-9_]+)', m.group(1))
    if not name or (len(sys.argv) > 2 and name.group(1) not in sys.argv[2:]):
        continue
    ins = [l.split()[0] for l in m.group(2).split('\n')
           if l.strip() and not l.strip().startswith((';', '.')) and not l.strip().endswith(':')]
    c = Counter(ins)
    waits = sum(v for k, v in c.items() if k == 's_waitcnt')
    print(f"{name.group(1):18s} n={len(ins):5d} ds_read={sum(v for k, v in c.items() if k.startswith('ds_read')):4d} "
          f"ds_write={sum(v for k, v in c.items() if k.startswith('ds_write')):3d} "
          f"ds_atomic={sum(v for k, v in c.items() if k.startswith('ds_add') or k.startswith('ds_max')):4d} "
          f"waitcnt={waits:4d} f64={sum(v for k, v in c.items() if 'f64' in k):5d} "
          f"gload={sum(v for k, v in c.items() if k.startswith('global_load')):3d} "
          f"scratch={sum(v for k, v in c.items() if k.startswith('scratch_')):3d}")

