#!/bin/bash
# Build tools/variants/lib_prev.so: exact_greedy.hip as committed at git revision $1 (default HEAD),
# the other objects from the regular build — the "previous build" side of an A/B call.
set -e
rev=${1:-HEAD}
cd "$(dirname "$0")/../vgposp_amd/csrc"
mkdir -p build/var ../../tools/variants
git show "$rev":vgposp_amd/csrc/exact_greedy.hip > build/var/exact_prevsrc.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I. -c build/var/exact_prevsrc.hip -o build/var/exact_prev.o
objs=$(ls build/*.o | grep -v '/exact_greedy.o')
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/var/exact_prev.o -o ../../tools/variants/lib_prev.so
echo built tools/variants/lib_prev.so from $rev
