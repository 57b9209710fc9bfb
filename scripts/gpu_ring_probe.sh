#!/bin/bash
# decode ring-depth probe: the split syn kernel alone (probe library, CLAY_DECODE_PROBE=13) at
# ring depths 10 / 8 / 7 (9 / 7 / 6 streaming buffers), 4-erasure (10,4,13) 1 GiB
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-ring}
for ring in ${RINGS:-10 8 7}; do
  CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_EXEC=stream CLAY_DECODE_PROBE=13 CLAY_DECODE_RING=$ring ONLY=decode timeout -k 10 120 python scripts/bench_paths.py > gpurun_out/${TAG}_r$ring.jsonl 2> gpurun_out/${TAG}_r$ring.err || { echo "ring $ring failed"; tail -5 gpurun_out/${TAG}_r$ring.err; exit 1; }
  echo "ring $ring (syn only)"; grep "0, 4, 8, 12" gpurun_out/${TAG}_r$ring.jsonl
done
