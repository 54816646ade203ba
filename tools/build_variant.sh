#!/bin/bash
# build/abl/libcpg_<name>.so with extra compile flags (development measurement only):
#   tools/build_variant.sh <name> "<flags>"
set -e
cd "$(dirname "$0")/../cpgisland_amd/csrc"
BASE='-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable --offload-arch=gfx950 -munsafe-fp-atomics'
mkdir -p ../../build/abl
make -s -j8 OBJDIR=../../build/abl/obj_$1 OUT=../../build/abl/libcpg_$1.so CXXFLAGS="$BASE $2" ../../build/abl/libcpg_$1.so
# a package tree that loads this variant: CPG_DEV_PKG=build/abl/pkg_<name> (tests/conftest.py
# and the tools put it first on sys.path); the product loader itself has no override
P=../../build/abl/pkg_$1/cpgisland_amd
rm -rf $P && mkdir -p $P
cp ../*.py $P/ && cp ../../build/abl/libcpg_$1.so $P/libcpg.so
[ -f ../libcpg_isl_timeout.so ] && cp ../libcpg_isl_timeout.so $P/
