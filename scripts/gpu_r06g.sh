#!/bin/bash
# Round 6: same-box A/B of library builds (CLAY_AMD_LIB) on (10,4,13) 1 GiB decodes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06g}; shift
for rep in 1 2; do
for L in ${LIBS:-libclay_amd.so}; do
  CLAY_AMD_LIB=$R/clay_amd/$L timeout -k 10 120 python scripts/time_decode.py "$@" >> gpurun_out/${TAG}.txt 2>&1 || { echo "$L failed"; tail -5 gpurun_out/${TAG}.txt; exit 1; }
done
done
cat gpurun_out/${TAG}.txt
