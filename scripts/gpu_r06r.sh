#!/bin/bash
# Round 6: TWO small patterns + 1 GiB two-in-section tests, (2,1) timings auto vs fused2, decode PMC.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06r}
echo "[$(date +%T)] tests"
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_stream_decode.py -m gpu -k "two_erasures or two_in_a_section_1GiB" > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] timings"
DATA_ONLY=1 timeout -k 10 200 python scripts/time_decode.py 0,1,4 0,4,5 12,13,0 13,1,2 0,1 0,1,2,3 > gpurun_out/${TAG}_auto.txt 2>&1 || { echo "time failed"; tail -5 gpurun_out/${TAG}_auto.txt; exit 1; }
cat gpurun_out/${TAG}_auto.txt
EXEC=stream-fused2 DATA_ONLY=1 timeout -k 10 200 python scripts/time_decode.py 0,1,4 0,4,5 12,13,0 13,1,2 0,1 > gpurun_out/${TAG}_f2.txt 2>&1 || { echo "time f2 failed"; tail -5 gpurun_out/${TAG}_f2.txt; exit 1; }
cat gpurun_out/${TAG}_f2.txt
echo "[$(date +%T)] decode PMC"
DATA_ONLY=1 bash scripts/pmc_decode.sh ${TAG}_pd_f2 && ER=0,1,4,8 DATA_ONLY=1 bash scripts/pmc_decode.sh ${TAG}_pd_two
echo "[$(date +%T)] done"
