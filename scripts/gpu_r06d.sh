#!/bin/bash
# Round 6: same-box A/B of the round-5 library encode (bench.py, short) against the probe's lane
# maps (stream_probe n8: map 0 = round-5 map with the round-6 register fixes, map 8, map 9).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06d}
echo "[$(date +%T)] bench (library)"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-host-path --no-small --no-legs --cpu-seconds 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
echo "[$(date +%T)] stream_probe n8"
timeout -k 10 240 ./bench_tools/stream_probe 419432 n8 > gpurun_out/${TAG}_n8.txt 2>&1 || { echo "probe failed rc=$?"; tail -20 gpurun_out/${TAG}_n8.txt; exit 1; }
cat gpurun_out/${TAG}_n8.txt
echo "[$(date +%T)] bench (library) again"
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-host-path --no-small --no-legs --cpu-seconds 1 > gpurun_out/${TAG}_bench2.json 2> gpurun_out/${TAG}_bench2.err || { echo "bench failed rc=$?"; tail -20 gpurun_out/${TAG}_bench2.err; exit 1; }
cat gpurun_out/${TAG}_bench2.json
