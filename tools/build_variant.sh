#!/bin/bash
# An A/B variant of libmbx built with extra compile flags, in a scratch copy
# of csrc (the production objects stay as they are):
#   tools/build_variant.sh NAME "-DFLAG=VALUE ..."  ->  minibase-columnar-database_amd/libmbx_NAME.so
# Load it with MBX_LIB=libmbx_NAME.so-path in tools that honour it (tools/c3_u_ab.py).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
FLAGS=$2
B=/tmp/mbx_variant_$NAME
rm -rf $B && mkdir -p $B/pkg/csrc $B/include
cp $ROOT/minibase-columnar-database_amd/csrc/*.hip $ROOT/minibase-columnar-database_amd/csrc/*.cpp \
   $ROOT/minibase-columnar-database_amd/csrc/*.hpp $ROOT/minibase-columnar-database_amd/csrc/Makefile $B/pkg/csrc/
cp $ROOT/include/*.h $B/include/
make -C $B/pkg/csrc -j4 OUT=$ROOT/minibase-columnar-database_amd/libmbx_$NAME.so \
     CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value $FLAGS" > $B/build.log 2>&1
echo "built $ROOT/minibase-columnar-database_amd/libmbx_$NAME.so"
