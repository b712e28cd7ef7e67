#!/bin/bash
# Build tools/variants/lib_NAME.so: the product gemm.hip with extra -D flags, linked with the other
# objects of the regular build (make -C vgposp_amd/csrc first).  Load it with VGPOSP_LIB=...
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c gemm.hip -o build/var/gemm_$name.o
objs=$(ls build/*.o | grep -v '/gemm.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/gemm_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
