#!/bin/bash
# Build E-step ablation variants of libcpg into build/abl/ (development measurement only).
set -e
cd "$(dirname "$0")/../cpgisland_amd/csrc"
BASE='-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics'
for v in dbgchain:"-DCPG_DEBUG_CHAIN"; do
  name=${v%%:*}; flags=${v#*:}
  make -s -j8 OBJDIR=../../build/abl/obj_$name OUT=../../build/abl/libcpg_$name.so CXXFLAGS="$BASE $flags"
done
ls -la ../../build/abl/*.so
