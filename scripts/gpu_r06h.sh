#!/bin/bash
# Round 6: k_stream_fused2 with two erasures in a section -- GPU tests, then timings.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06h}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
echo "[$(date +%T)] pytest two-in-a-section"
timeout -k 10 600 $PYT tests/test_gpu_stream_decode.py -m gpu -k "two_erasures" > gpurun_out/${TAG}_pytest_two.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_pytest_two.log | tail -30; exit 1; }
tail -2 gpurun_out/${TAG}_pytest_two.log
echo "[$(date +%T)] pytest stream decode (all)"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stream_decode.py tests/test_gpu_stream_local.py tests/test_gpu_codeword_decode.py -m gpu > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] timings"
timeout -k 10 300 python scripts/time_decode.py 0,4,8,12 0,4,8 4,13 0,1,4,8 0,1,4,12 0,1,4,5 8,9,0,4 0,8,9,10 > gpurun_out/${TAG}_time.txt 2>&1 || { echo "time failed"; tail -5 gpurun_out/${TAG}_time.txt; exit 1; }
cat gpurun_out/${TAG}_time.txt
echo "[$(date +%T)] done"
