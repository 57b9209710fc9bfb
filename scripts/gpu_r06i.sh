#!/bin/bash
# Round 6: fused2 region layout A/B (swizzled vs plain) on the same box: kernel times of the
# decode patterns, then the probe libraries' segment timing (PROBE 40) and part-skipping probes.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06i}
P="0,4,8,12 0,1,4,8 0,1,4,5 0,8,9,10"
for rep in 1 2; do
for L in libclay_amd.so libclay_amd_sw0.so; do
  CLAY_AMD_LIB=$R/clay_amd/$L timeout -k 10 120 python scripts/time_decode.py $P >> gpurun_out/${TAG}.txt 2>&1 || { echo "$L failed"; tail -5 gpurun_out/${TAG}.txt; exit 1; }
done
done
for L in libclay_amd_p1.so libclay_amd_p0.so; do
  for PR in 40 31 35 34; do
    echo "== $L probe $PR" >> gpurun_out/${TAG}.txt
    CLAY_DECODE_PROBE=$PR CLAY_AMD_LIB=$R/clay_amd/$L timeout -k 10 120 python scripts/time_decode.py 0,4,8,12 0,1,4,8 >> gpurun_out/${TAG}.txt 2>&1 || { echo "$L $PR failed"; tail -5 gpurun_out/${TAG}.txt; exit 1; }
  done
done
grep -v amdgpu.ids gpurun_out/${TAG}.txt | grep -v "^f2-timing" ; grep "^f2-timing" gpurun_out/${TAG}.txt | sort | uniq -c | sort -rn | head -8
