#!/bin/bash
# local decode check on the GPU box: parity tests of the local decodes, then (10,4,13) 1 GiB path
# timings of the 256-byte-run kernel and (CLAY_LOCAL_W64=1) the 64-byte-tile kernel
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-lc}
echo "[$(date +%T)] local decode tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream_local.py tests/test_gpu_codeword_decode.py ${EXTRA_TESTS} > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] paths"
ONLY=local RUNS=${RUNS:-10} timeout -k 10 180 python scripts/bench_paths.py > gpurun_out/${TAG}_paths.jsonl 2> gpurun_out/${TAG}_paths.err || { echo "paths failed"; tail -5 gpurun_out/${TAG}_paths.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_paths.jsonl
CLAY_LOCAL_W64=1 ONLY=local RUNS=${RUNS:-10} timeout -k 10 180 python scripts/bench_paths.py > gpurun_out/${TAG}_paths_w64.jsonl 2> gpurun_out/${TAG}_paths_w64.err || { echo "paths w64 failed"; tail -5 gpurun_out/${TAG}_paths_w64.err; exit 1; }
cut -c1-220 gpurun_out/${TAG}_paths_w64.jsonl
