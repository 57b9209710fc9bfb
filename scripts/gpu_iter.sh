#!/bin/bash
# GPU iteration: targeted parity tests (PYTEST_K), an optional probe binary, then a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-iter}
K=${PYTEST_K:-"stream"}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -x -q -k "$K" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -n 2 gpurun_out/${TAG}_pytest.log
if [ -n "$PROBE" ]; then
  timeout -k 10 300 $PROBE > gpurun_out/${TAG}_probe.txt 2>&1 || { echo "probe failed"; tail -20 gpurun_out/${TAG}_probe.txt; exit 1; }
  cat gpurun_out/${TAG}_probe.txt
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-host-path --no-small --cpu-seconds 0 > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
python - "$R/gpurun_out/${TAG}_bench.log" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print("bench", d["config"]["encode_path"], "ms_mean", d["roofline"]["kernel_ms_mean"], "min", d["roofline"]["kernel_ms_min"], "frac", d["roofline"]["frac"])
PY
