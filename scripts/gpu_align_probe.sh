#!/bin/bash
# encode row / tile alignment A/B (bench_tools/stream_probe a): the BASELINE sub-chunk 419,432
# (row starts at 104 * z mod 128) and 419,456 (128-aligned rows), XCD regions rounded to 32 B
# (the library) or 256 B (every tile 256-byte aligned within its row)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-al}
for cfg in "419432 32" "419456 256" "419456 32" "419432 256"; do
  set -- $cfg
  timeout -k 10 120 ./bench_tools/stream_probe $1 a $2 >> gpurun_out/${TAG}.txt 2>&1 || { echo "probe $cfg failed"; tail -5 gpurun_out/${TAG}.txt; exit 1; }
done
cat gpurun_out/${TAG}.txt
