#!/bin/bash
# build/abl/libcpg_<name>.so from the sources of a git revision (development measurement only:
# the A side of an A/B against the working tree), with its package tree for CPG_DEV_PKG:
#   tools/build_rev.sh <name> <rev>
set -e
NAME=$1; REV=$2
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC=$ROOT/build/abl/src_$NAME
rm -rf $SRC && mkdir -p $SRC
git -C $ROOT archive $REV cpgisland_amd include | tar -x -C $SRC
BASE='-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics'
make -s -j8 -C $SRC/cpgisland_amd/csrc OBJDIR=$ROOT/build/abl/obj_$NAME \
     OUT=$ROOT/build/abl/libcpg_$NAME.so CXXFLAGS="$BASE" $ROOT/build/abl/libcpg_$NAME.so
P=$ROOT/build/abl/pkg_$NAME/cpgisland_amd
rm -rf $P && mkdir -p $P
cp $SRC/cpgisland_amd/*.py $P/ && cp $ROOT/build/abl/libcpg_$NAME.so $P/libcpg.so
# host-side helpers the tree's tools import that the revision lacks (e.g. fingerprint.py)
for f in $ROOT/cpgisland_amd/*.py; do [ -f $P/$(basename $f) ] || cp $f $P/; done
echo "built $ROOT/build/abl/libcpg_$NAME.so from $REV"
