#!/bin/bash
# Round 6: k_bs_decode1 ((4,2,5) single erasure) tests + cfg2 timing; fused2 data-only timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06o}
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
echo "[$(date +%T)] pytest decode1"
timeout -k 10 300 $PYT tests/test_gpu_line_kernels.py tests/test_gpu_parity.py -k "decode1 or encode1 or small_decode_plan or bitsliced_encode" -m gpu > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "pytest failed rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/${TAG}_pytest.log
echo "[$(date +%T)] cfg2 + cfg5 timings"
timeout -k 10 300 env ONLY=cfg2,c2e python scripts/bench_paths.py > gpurun_out/${TAG}_cfg2.txt 2>&1 || { echo "cfg2 failed"; tail -5 gpurun_out/${TAG}_cfg2.txt; exit 1; }
cat gpurun_out/${TAG}_cfg2.txt
CLAY_EXEC=tile timeout -k 10 300 env ONLY=cfg2,c2e python scripts/bench_paths.py > gpurun_out/${TAG}_cfg2_tile.txt 2>&1 || { echo "cfg2 tile failed"; tail -5 gpurun_out/${TAG}_cfg2_tile.txt; exit 1; }
cat gpurun_out/${TAG}_cfg2_tile.txt
DATA_ONLY=1 timeout -k 10 300 python scripts/time_decode.py 0,4,8,12 0,1,4,8 > gpurun_out/${TAG}_f2data.txt 2>&1 || { echo "time failed"; tail -5 gpurun_out/${TAG}_f2data.txt; exit 1; }
cat gpurun_out/${TAG}_f2data.txt
echo "[$(date +%T)] done"
