#!/bin/bash
# Build tools/variants/lib_NAME.so: the product exact_greedy.hip with extra -D flags, the other
# objects from the regular build (make -C vgposp_amd/csrc first).  Load it with
# VGPOSP_LIB=$PWD/tools/variants/lib_NAME.so (A/B timing only).  SRC=../../tools/variants/exact_greedy_dbg.hip
# with -DVGPOSP_EXACT_DBG=1|2|3: the phase-stamped copy that tools/exact_dbg.py reads.
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I. "$@" -c "${SRC:-exact_greedy.hip}" -o build/var/exact_$name.o
objs=$(ls build/*.o | grep -v '/exact_greedy.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/exact_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
