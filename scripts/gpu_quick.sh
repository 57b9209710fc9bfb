#!/bin/bash
# quick GPU iteration: targeted tests + one-process sweep
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-quick}; shift
K=${PYTEST_K:-"bitsliced or encode"}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m "gpu and not slow" -x -q -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python scripts/sweep_encode.py "$@" > gpurun_out/${TAG}_sweep.json 2>gpurun_out/${TAG}_sweep.err || { echo "sweep failed"; tail -20 gpurun_out/${TAG}_sweep.err; exit 1; }
cat gpurun_out/${TAG}_sweep.json
