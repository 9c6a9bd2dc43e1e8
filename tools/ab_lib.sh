#!/bin/bash
# Build an A/B variant of librcdc.so from the same sources with extra
# defines, into rustic_core_amd/ab/<name>.so (git-ignored; it travels to the
# GPU box with the tree).  Load it with RCDC_LIB=rustic_core_amd/ab/<name>.so.
# usage: tools/ab_lib.sh NAME -DFLAG ...
set -e
NAME=$1; shift
cd "$(dirname "$0")/../rustic_core_amd/csrc"
mkdir -p ../ab
make -s OUT=../ab/$NAME.so OBJDIR=../../build/ab_$NAME HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*" ../ab/$NAME.so
echo "built rustic_core_amd/ab/$NAME.so"
