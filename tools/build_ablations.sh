#!/bin/bash
# Build ablation variants of libcpg into build/abl/ (development measurement only).
set -e
cd "$(dirname "$0")/../cpgisland_amd/csrc"
BASE='-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics'
VARIANTS=${VARIANTS:-"kd0r64:-DEST_KD=0 -DEST_REP=64 kd1r64:-DEST_KD=1 -DEST_REP=64 kd0r72:-DEST_KD=0 -DEST_REP=72 kd1r80:-DEST_KD=1 -DEST_REP=80"}
rm -rf ../../build/abl/*.so
for v in $VARIANTS; do :; done
python3 - "$VARIANTS" <<'PY' > /tmp/abl_list
import sys
toks = sys.argv[1].split()
out = []; cur = None
for t in toks:
    if ':' in t and not t.startswith('-'):
        cur = t.split(':', 1); out.append([cur[0], cur[1]])
    else:
        out[-1][1] += ' ' + t
for n, f in out: print(n + '|' + f)
PY
while IFS='|' read -r name flags; do
  make -s -j8 OBJDIR=../../build/abl/obj_$name OUT=../../build/abl/libcpg_$name.so CXXFLAGS="$BASE $flags"
done < /tmp/abl_list
ls -la ../../build/abl/*.so
