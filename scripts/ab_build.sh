#!/bin/bash
# Build a variant of libquadtrack.so for a same-box A/B (run here, after `make`):
#   bash scripts/ab_build.sh NAME "DEFS" TU...
# copies the in-tree objects to build/ab/NAME/obj, rebuilds the named
# translation units (e.g. qt_rollout) with DEFS (e.g. -DQT_EXACT_VPIN=0) and
# links build/ab/NAME/libquadtrack.so.  A GPU run selects it with
# QUADTRACK_LIB=$PWD/build/ab/NAME/libquadtrack.so.
set -e
cd "$(dirname "$0")/.."
name=$1; defs=$2; shift 2
d=build/ab/$name
mkdir -p $d/obj
cp lqr-quadcopter-test_amd/build/*.o $d/obj/
for tu in "$@"; do rm -f $d/obj/$tu.o; done
make -s -C lqr-quadcopter-test_amd OBJ=$PWD/$d/obj OUT=$PWD/$d DEFS="$defs" -j4
ls -la $d/libquadtrack.so
