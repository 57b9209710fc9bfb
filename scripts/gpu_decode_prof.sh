#!/bin/bash
# Kernel trace of the (10,4,13) 1 GiB 4-erasure decode {0,4,8,12} (scripts/prof_decode.py) under
# the executor CLAY_EXEC (default stream: the local decode or the fused decode v2).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-dprof}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
CLAY_EXEC=${CLAY_EXEC:-stream} timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/trace" -o t -- python3 "$R/scripts/prof_decode.py" --what decode4 --iters 20 > "$R/gpurun_out/$TAG/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/$TAG/trace.log"; exit 1; }
find "$R/gpurun_out/$TAG/trace" -type f ! -name "*stats*" -delete
cut -c1-160 "$R"/gpurun_out/$TAG/trace/*kernel_stats.csv
