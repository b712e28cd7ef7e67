#!/bin/bash
# Round 4, final evidence on the final build: GPU tests + smoke + the default bench line
# (tools/round_end.sh), then the round-4 profiles (tools/profile_r4.sh).
set -e
R=${GRAFT_REPO_ROOT:-$PWD}
bash $R/tools/round_end.sh
bash $R/tools/profile_r4.sh
