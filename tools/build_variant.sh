#!/bin/bash
# Build tools/variants/lib_NAME.so: tools/variants/gemm_experiments.hip (the product gemm.hip plus
# the measured-and-rejected variants) with extra -D flags, the other objects from the
# regular build (make -C vgposp_amd/csrc first).  Load it with VGPOSP_LIB=$PWD/tools/variants/...
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 "$@" -c ../../tools/variants/gemm_experiments.hip -o build/var/gemm_$name.o
objs=$(ls build/*.o | grep -v '/gemm.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/gemm_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
