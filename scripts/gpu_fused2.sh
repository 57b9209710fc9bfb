#!/bin/bash
# fused decode v2: its parity tests, then the 4-erasure (10,4,13) 1 GiB timing and the probe
# breakdown (CLAY_DECODE_PROBE 31 no rounds, 32 no stores, 34 no phase-A math, 35 memory only)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-f2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_decode.py -x -q -k fused2 --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for pr in ${PROBES:-0 31 32 34 35}; do
  CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_EXEC=stream-fused2 CLAY_DECODE_PROBE=$pr ONLY=decode timeout -k 10 120 python scripts/bench_paths.py > gpurun_out/${TAG}_p$pr.jsonl 2> gpurun_out/${TAG}_p$pr.err || { echo "probe $pr failed"; tail -5 gpurun_out/${TAG}_p$pr.err; exit 1; }
  echo "probe $pr"; grep "0, 4, 8, 12" gpurun_out/${TAG}_p$pr.jsonl
done
