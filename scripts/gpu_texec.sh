#!/bin/bash
# GPU iteration for the plan executors: targeted parity tests (PYTEST_K), then the
# decode/repair path timings under the tile-fused and the grouped executor.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-texec}
K=${PYTEST_K:-"decode or repair or tile or exec"}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -x -q -k "$K" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_pytest.log
for mode in ${MODES:-tile grouped}; do
  big=0; ex=$mode; if [ "$mode" = tilebig ]; then big=1; ex=tile; fi
  CLAY_TEXEC_BIG=$big CLAY_EXEC=$ex ONLY=${ONLY:-decode,repair} timeout -k 10 300 python scripts/bench_paths.py > gpurun_out/${TAG}_paths_${mode}.jsonl 2> gpurun_out/${TAG}_paths_${mode}.err || { echo "paths $mode failed"; tail -20 gpurun_out/${TAG}_paths_${mode}.err; exit 1; }
  python - "$R/gpurun_out/${TAG}_paths_${mode}.jsonl" "$mode" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[2], d["config"], d["median_ms"], "ms", d["frac_of_8TBps"], d["path"], d["launches"])
PY
done
