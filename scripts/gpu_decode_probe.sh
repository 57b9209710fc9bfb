#!/bin/bash
# streaming-decode tests + probe breakdown (CLAY_DECODE_PROBE: 1 no phase B, 2 no phase-A math,
# 3 neither, 7 neither and no DMA)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-dprobe}
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for pr in ${PROBES:-0 1 2 3 7}; do
  CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_EXEC=stream CLAY_DECODE_PROBE=$pr ONLY=decode timeout -k 10 120 python scripts/bench_paths.py > gpurun_out/${TAG}_p$pr.jsonl 2> gpurun_out/${TAG}_p$pr.err || { echo "probe $pr failed"; tail -5 gpurun_out/${TAG}_p$pr.err; exit 1; }
  echo "probe $pr"; grep -v "(4,2,5)" gpurun_out/${TAG}_p$pr.jsonl | python3 -c "import sys,json; [print(' ', json.loads(l)['config'], json.loads(l)['median_ms'], json.loads(l)['path']) for l in sys.stdin]"
done
