#!/bin/bash
# A -DMBX_DIAG build of libmbx (the A/B-only kernel forms kept) into
# minibase-columnar-database_amd/libmbx_diag.so, built in a scratch copy of
# csrc so the production objects stay as they are.  For tools/c2_anatomy.py.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=/tmp/mbx_diag_build
rm -rf $B && mkdir -p $B/pkg/csrc $B/include
cp $ROOT/minibase-columnar-database_amd/csrc/*.hip $ROOT/minibase-columnar-database_amd/csrc/*.cpp \
   $ROOT/minibase-columnar-database_amd/csrc/*.hpp $ROOT/minibase-columnar-database_amd/csrc/Makefile $B/pkg/csrc/
cp $ROOT/include/*.h $B/include/
make -C $B/pkg/csrc -j8 OUT=$ROOT/minibase-columnar-database_amd/libmbx_diag.so \
     CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value -DMBX_DIAG" > $B/build.log 2>&1
echo "built $ROOT/minibase-columnar-database_amd/libmbx_diag.so"
