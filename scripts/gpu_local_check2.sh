#!/bin/bash
# local decode parity (incl. sub-chunks that are not multiples of 8) and path timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-lc}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream_local.py tests/test_gpu_codeword_decode.py tests/test_gpu_stream_decode.py > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
ONLY=local RUNS=10 timeout -k 10 200 python scripts/bench_paths.py > gpurun_out/${TAG}_paths.jsonl 2> gpurun_out/${TAG}_paths.err || { echo "paths failed"; tail -5 gpurun_out/${TAG}_paths.err; exit 1; }
cut -c1-200 gpurun_out/${TAG}_paths.jsonl
