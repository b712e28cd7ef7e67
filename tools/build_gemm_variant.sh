#!/bin/bash
# Build tools/variants/lib_NAME.so: the product gemm.hip (or SRC=path/to/gemm_variant.hip) with
# extra -D flags, linked with the other objects of the regular build (make -C vgposp_amd/csrc
# first).  Load it with VGPOSP_LIB=...  Round 6's loop experiments:
#   SRC=../../tools/variants/gemm_r6_pipe.hip tools/build_gemm_variant.sh pipe -DVGPOSP_GEMM_PIPE=1
#   (further switches: -DVGPOSP_GEMM_SPREAD=1|2, -DVGPOSP_GEMM_CFG=4, and the timing-only
#   -DVGPOSP_GEMM_EXP_NOLOAD / _NOBAR / _FIXADDR; profiles/r6_gemm_ab.jsonl)
set -e
name=$1; shift
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p ../../tools/variants build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I. "$@" -c "${SRC:-gemm.hip}" -o build/var/gemm_$name.o
objs=$(ls build/*.o | grep -v '/gemm.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/gemm_$name.o -o ../../tools/variants/lib_$name.so
echo built tools/variants/lib_$name.so
