#!/bin/bash
# Build tools/variants/lib_NAME.so: the product exact_greedy.hip with extra -D flags, the other
# objects from the regular build (make -C vgposp_amd/csrc first).  Load it with
# VGPOSP_LIB=$PWD/tools/variants/lib_NAME.so (A/B timing only).
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c exact_greedy.hip -o build/var/exact_$name.o
objs=$(ls build/*.o | grep -v '/exact_greedy.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/exact_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
