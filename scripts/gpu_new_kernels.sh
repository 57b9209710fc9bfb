#!/bin/bash
# new single-launch kernels: their parity tests, the capture test, then path timings
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-nk}
timeout -k 10 400 python -u -m pytest tests/test_gpu_repair_kernel.py tests/test_gpu_stream_decode.py tests/test_gpu_runtime.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
for ex in stream auto; do
  CLAY_EXEC=$ex ONLY=${ONLY:-decode,repair} timeout -k 10 200 python scripts/bench_paths.py > gpurun_out/${TAG}_paths_$ex.jsonl 2> gpurun_out/${TAG}_paths_$ex.err || { echo "paths $ex failed"; tail -5 gpurun_out/${TAG}_paths_$ex.err; exit 1; }
  echo "exec $ex"; python3 -c "import sys,json; [print(' ', (d:=json.loads(l))['config'], d['median_ms'], d['frac_of_8TBps'], d['path']) for l in open(sys.argv[1])]" gpurun_out/${TAG}_paths_$ex.jsonl
done
