#!/bin/bash
# Build tools/variants/lib_NAME.so: the product potrf.hip with extra -D flags (e.g. -DVGPOSP_STAMPS),
# the other objects from the regular build.  Load it with VGPOSP_LIB=$PWD/tools/variants/lib_NAME.so.
# SRC=../../tools/variants/potrf_stamps.hip: the phase-stamped copy (-DVGPOSP_STAMPS).
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I. "$@" -c "${SRC:-potrf.hip}" -o build/var/potrf_$name.o
objs=$(ls build/*.o | grep -v '/potrf.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/potrf_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
