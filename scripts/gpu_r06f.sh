#!/bin/bash
# Round 6: fused decode v2 with the swizzled S/C region: its GPU tests, the config legs, and the
# PMC passes of the {0,4,8,12} decode (bank conflicts, traffic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06f}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
echo "[$(date +%T)] pytest stream decode + cfg5"
timeout -k 10 600 $PYT tests/test_gpu_stream_decode.py tests/test_gpu_parity.py -m gpu -k "fused2 or cfg5 or stream_decode or decode" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] legs"
timeout -k 10 300 python scripts/legs_only.py > gpurun_out/${TAG}_legs.txt 2>&1 || { echo "legs failed rc=$?"; tail -20 gpurun_out/${TAG}_legs.txt; exit 1; }
cat gpurun_out/${TAG}_legs.txt
echo "[$(date +%T)] pmc decode"
bash scripts/pmc_decode.sh ${TAG}_pmc || exit 1
echo "[$(date +%T)] done"
