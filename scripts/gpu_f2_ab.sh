#!/bin/bash
# fused2 A/B on the probe library, then the decode GPU tests (fused2 / local / config 5 / the
# full-size local256 tests) on the product library
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-ab}
PROBES="${PROBES:-0 45 0 45}" bash scripts/gpu_fused2_probe.sh ${TAG} || exit 1
echo "[$(date +%T)] decode tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stream_decode.py tests/test_gpu_parity.py -m gpu -k "${TESTK:-fused2 or local256 or cfg5 or stream}" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
