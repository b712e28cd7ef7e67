#!/bin/bash
# rocprofv3 kernel stats of tools/b512_probe.py for the in-tree library and the given variants.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/b512p
mkdir -p $O
for lib in default "$@"; do
  tag=$(basename "$lib" .so)
  if [[ $lib == default ]]; then unset VGPOSP_LIB; else export VGPOSP_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- python3 -u tools/b512_probe.py > $O/probe_$tag.log 2>&1
  echo "$tag: $(grep -h 'potrf ms\|max rel' $O/probe_$tag.log | tr '\n' ' ')"
  f=$(find $O/prof_$tag -name '*kernel_stats.csv' | head -1)
  grep -h "block512\|potrf_leaf\|gemm_glds" "$f" | cut -c1-160 | head -6
done
