#!/bin/bash
# Same-box A/B of two library builds on decode patterns: alternating runs of scripts/time_decode.py
# with CLAY_AMD_LIB = clay_amd/$1 and clay_amd/$2 (default the shipping library), 3 rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
A=${1:-libclay_amd_old.so}; B=${2:-libclay_amd.so}; TAG=${TAG:-ab}
PATS=${PATS:-"0,4,8,12 0,1,4,8 0,1,4,5 8,9,0,4 0,4,8"}
for i in 1 2 3; do
  for L in $A $B; do
    CLAY_AMD_LIB=$R/clay_amd/$L DATA_ONLY=1 timeout -k 10 200 python scripts/time_decode.py $PATS >> gpurun_out/${TAG}.txt 2>&1 || { echo "run $L failed"; tail -5 gpurun_out/${TAG}.txt; exit 1; }
  done
done
grep median gpurun_out/${TAG}.txt
