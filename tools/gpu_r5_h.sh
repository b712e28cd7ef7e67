#!/bin/bash
# Round 5, call H: the step kernel's key-refresh phases (-DVGPOSP_EXACT_DBG=2 build).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
O=$R/gpurun_out/r5h
mkdir -p $O
cd $R
VGPOSP_LIB=$R/tools/variants/lib_dbg2.so timeout -k 10 120 python -u tools/exact_dbg.py --dbg2 > $O/c4_dbg2.json 2>&1
echo ok dbg2
