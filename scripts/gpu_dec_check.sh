#!/bin/bash
# decode check on the GPU box: fused2 probes (probe library) then the decode GPU tests (product library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-dc}
PROBES="${PROBES:-0 43}" bash scripts/gpu_fused2_probe.sh ${TAG} || exit 1
echo "[$(date +%T)] decode tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "${TESTK:-decode or fused2 or codeword}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
