#!/bin/bash
# Kernel trace + HBM PMC passes (one counter per rocprofv3 run) of the (4,2,5) line-local kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-pmc_cfg2}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$TAG/trace" -o p -- python3 "$R/scripts/prof_cfg2.py" --iters 50 > "$R/gpurun_out/$TAG/trace.log" 2>&1 || { echo "trace failed"; tail -5 "$R/gpurun_out/$TAG/trace.log"; exit 1; }
for n in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $n --output-format csv -d "$R/gpurun_out/$TAG/$n" -o p -- python3 "$R/scripts/prof_cfg2.py" --iters 4 > "$R/gpurun_out/$TAG/$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$R/gpurun_out/$TAG/$n.log"; exit 1; }
done
find "$R/gpurun_out/$TAG" -name "*kernel_stats*"
echo "pmc done"
