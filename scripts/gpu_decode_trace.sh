#!/bin/bash
# rocprofv3 kernel traces of the (10,4,13) 1 GiB decodes after a 250 ms prewarm, 300 measured
# launches each: {0,4,8,12} (fused decode v2), {0} and {0,4} (local decode, 256-byte runs);
# summaries over the measured launches only (scripts/trace_summary.py --skip <prewarm calls>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-dtr}
mkdir -p "$R/gpurun_out/$TAG"
export TMPDIR=/tmp
for er in ${ERS:-0,4,8,12 0 0,4}; do
  n=$(echo $er | tr , _)
  ( cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/$TAG/e$n" -o t -- python3 "$R/scripts/prof_decode.py" --er $er --iters 300 --prewarm-ms 250 ) > "$R/gpurun_out/$TAG/e$n.log" 2>&1 || { echo "trace $er failed"; tail -5 "$R/gpurun_out/$TAG/e$n.log"; exit 1; }
  w=$(grep -o "prewarm_calls [0-9]*" "$R/gpurun_out/$TAG/e$n.log" | awk '{print $2}')
  f=$(find "$R/gpurun_out/$TAG/e$n" -name "*kernel_trace.csv" | head -1)
  python3 "$R/scripts/trace_summary.py" "$f" k_stream --skip $w | tee "$R/gpurun_out/$TAG/e${n}_summary.json"
  rm -f "$f"
done
