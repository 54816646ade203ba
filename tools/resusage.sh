#!/bin/bash
# Per-kernel VGPRs / spills / occupancy of one HIP source (dev tool):
#   tools/resusage.sh k_estep.hip [extra hipcc flags]
cd "$(dirname "$0")/../cpgisland_amd/csrc"
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off --offload-arch=gfx950 -munsafe-fp-atomics \
  "$@" -x hip -c "$f" -o /tmp/resusage.o -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c "
import re, sys
cur = None; rows = {}
for line in sys.stdin:
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = m.group(1); rows[cur] = {}; continue
    m = re.search(r'remark:\s+([A-Za-z /\[\]]+?):\s+(\S+)', line)
    if m and cur: rows[cur][m.group(1).strip()] = m.group(2)
for k, v in rows.items():
    n = re.search(r'(k_[a-z0-9_]+)', k); n = n.group(1) if n else k[:40]
    tpl = re.search(r'ILb(\d)EL?b?(\d)?', k)
    print(f\"{n:24s} {k[-30:]:30s} vgpr={v.get('VGPRs','?'):>4} spill={v.get('VGPRs Spill','?'):>3} occ={v.get('Occupancy [waves/SIMD]','?')}\")
"
