#!/bin/bash
# Round 4, call O: the round-4 profiles (C4 stats and PMC first, the 65k step's GEMM PMC last).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/tools/profile_r4.sh
