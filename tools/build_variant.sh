#!/bin/bash
# build/abl/libcpg_<name>.so from a PATCHED copy of the sources (development measurement only;
# the product sources carry no build-time knobs):
#   tools/build_variant.sh <name> "<extra flags>" ['<file>:<sed expression>' | '<file>:@<script.py>' ...]
# e.g. tools/build_variant.sh grid4k "" 'k_count.hip:s/kCntGrid = 2048/kCntGrid = 4096/'
# Every expression must change its file (checked), so a stale patch fails loudly.
set -e
NAME=$1; FLAGS=$2; shift 2
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
SRC=$ROOT/build/abl/src_$NAME
rm -rf $SRC && mkdir -p $SRC/csrc $SRC/include
cp $ROOT/cpgisland_amd/csrc/*.hip $ROOT/cpgisland_amd/csrc/*.cpp $ROOT/cpgisland_amd/csrc/*.h \
   $ROOT/cpgisland_amd/csrc/Makefile $SRC/csrc/
cp $ROOT/include/cpg.h $SRC/include/
# the Makefile names ../../include/cpg.h: keep that depth
for p in "$@"; do
  f=${p%%:*}; e=${p#*:}
  cp $SRC/csrc/$f $SRC/csrc/$f.orig
  # '<file>:@<script.py>': the script rewrites the file in place (multi-line edits)
  if [ "${e:0:1}" = "@" ]; then python3 ${e:1} $SRC/csrc/$f; else sed -i -e "$e" $SRC/csrc/$f; fi
  if cmp -s $SRC/csrc/$f $SRC/csrc/$f.orig; then echo "patch changed nothing: $p" >&2; exit 1; fi
  rm $SRC/csrc/$f.orig
done
sed -i 's#\.\./\.\./include/cpg\.h#../include/cpg.h#' $SRC/csrc/Makefile
sed -i 's#"\.\./\.\./include/cpg\.h"#"../include/cpg.h"#' $SRC/csrc/*.h $SRC/csrc/*.hip $SRC/csrc/*.cpp 2>/dev/null || true
BASE='-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics'
mkdir -p $ROOT/build/abl
make -s -j8 -C $SRC/csrc OBJDIR=$ROOT/build/abl/obj_$NAME OUT=$ROOT/build/abl/libcpg_$NAME.so \
     CXXFLAGS="$BASE $FLAGS" $ROOT/build/abl/libcpg_$NAME.so
# a package tree that loads this variant: CPG_DEV_PKG=build/abl/pkg_<name> (tests/conftest.py
# and the tools put it first on sys.path); the product loader itself has no override
P=$ROOT/build/abl/pkg_$NAME/cpgisland_amd
rm -rf $P && mkdir -p $P
cp $ROOT/cpgisland_amd/*.py $P/ && cp $ROOT/build/abl/libcpg_$NAME.so $P/libcpg.so
echo "built $ROOT/build/abl/libcpg_$NAME.so"
