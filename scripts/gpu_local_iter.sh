#!/bin/bash
# local-decode iteration: its parity tests, then decode path timings (auto) and the grouped
# executor on the same patterns for comparison
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-loc}
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream_local.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
ONLY=${ONLY:-decode,decode23,decodeL} timeout -k 10 300 python scripts/bench_paths.py > gpurun_out/${TAG}_paths.jsonl 2> gpurun_out/${TAG}_paths.err || { echo "paths failed"; tail -20 gpurun_out/${TAG}_paths.err; exit 1; }
cat gpurun_out/${TAG}_paths.jsonl
if [ -n "$GROUPED" ]; then
CLAY_EXEC=grouped ONLY=decode23,decodeL timeout -k 10 300 python scripts/bench_paths.py > gpurun_out/${TAG}_paths_grouped.jsonl 2> gpurun_out/${TAG}_paths_grouped.err || { echo "grouped paths failed"; exit 1; }
cat gpurun_out/${TAG}_paths_grouped.jsonl
fi
