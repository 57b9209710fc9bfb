#!/bin/bash
# measurement probes: streaming-encode breakdown (quick set) and the bandwidth ceilings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-probes}
timeout -k 10 200 ./bench_tools/stream_probe 419432 q > gpurun_out/${TAG}_stream_probe.txt 2>&1 || { echo "stream_probe failed"; tail -5 gpurun_out/${TAG}_stream_probe.txt; exit 1; }
cat gpurun_out/${TAG}_stream_probe.txt
timeout -k 10 300 ./bench_tools/bw_probe > gpurun_out/${TAG}_bw_probe.txt 2>&1 || { echo "bw_probe failed"; tail -5 gpurun_out/${TAG}_bw_probe.txt; exit 1; }
cat gpurun_out/${TAG}_bw_probe.txt
