#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) and HBM bytes (FETCH_SIZE / WRITE_SIZE, one
# counter per pass) of the (9,3,11) repair of node 0, chunk 268,435,458 (scripts/prof_decode.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-rprof}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/trace" -o t -- python3 "$R/scripts/prof_decode.py" --what repair --iters 20 > "$R/gpurun_out/$TAG/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/$TAG/trace.log"; exit 1; }
find "$R/gpurun_out/$TAG/trace" -type f ! -name "*stats*" -delete
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d "$R/gpurun_out/$TAG/repair_$ctr" -o p -- python3 "$R/scripts/prof_decode.py" --what repair --iters 4 > "$R/gpurun_out/$TAG/repair_$ctr.log" 2>&1 || { echo "pmc $ctr failed"; tail -5 "$R/gpurun_out/$TAG/repair_$ctr.log"; exit 1; }
done
find "$R/gpurun_out/$TAG" -name "*stats*" -o -name "*counter_collection*"
