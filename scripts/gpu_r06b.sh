#!/bin/bash
# Round 6: lane-map A/B of the streaming encode (stream_probe n / nt).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06b}
for m in ${MODES:-n nt}; do
  echo "[$(date +%T)] stream_probe $m"
  timeout -k 10 240 ./bench_tools/stream_probe 419432 $m > gpurun_out/${TAG}_$m.txt 2>&1 || { echo "probe $m failed rc=$?"; tail -20 gpurun_out/${TAG}_$m.txt; exit 1; }
  cat gpurun_out/${TAG}_$m.txt
done
