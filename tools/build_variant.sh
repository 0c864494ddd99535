#!/bin/bash
# Build a compile-time variant of the library for A/B runs: syzkaller_amd/libsyzgpu_TAG.so from the same
# sources with extra -D flags (objects in syzkaller_amd/build_v/TAG). Load it with SYZGPU_LIB=<path>.
# Usage: bash tools/build_variant.sh TAG "-DSYZ_X=1 -DSYZ_Y=2"
set -e
TAG=$1; DEFS=$2
cd "$(dirname "$0")/../syzkaller_amd"
make -s -j8 BUILD=build_v/$TAG HIPFLAGS_EXTRA="$DEFS" LIB=libsyzgpu_$TAG.so variant
