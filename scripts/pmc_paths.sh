#!/bin/bash
# HBM bytes (FETCH_SIZE / WRITE_SIZE, one counter per rocprofv3 pass) of the decode-4 and
# repair paths (scripts/prof_decode.py), for the traffic-vs-algorithmic ratio.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmcp}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
for what in ${WHATS:-repair decode4}; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/$TAG/${what}_$ctr" -o p -- python3 "$R/scripts/prof_decode.py" --what $what --iters 4 > "$R/gpurun_out/$TAG/${what}_$ctr.log" 2>&1 || { echo "pmc $what $ctr failed"; tail -5 "$R/gpurun_out/$TAG/${what}_$ctr.log"; exit 1; }
  done
done
find "$R/gpurun_out/$TAG" -name "*counter_collection*" | head
