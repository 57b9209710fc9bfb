#!/bin/bash
# round-4 GPU pass: new kernels' parity tests + timings, then the full check (gpu_check.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r4}
echo "[$(date +%T)] local decode"
GROUPED=1 bash scripts/gpu_local_iter.sh ${TAG}_loc || exit 1
echo "[$(date +%T)] fused decode v2"
PROBES="0 31 35" bash scripts/gpu_fused2.sh ${TAG}_f2 || exit 1
echo "[$(date +%T)] (9,3) stream encode"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k stream3 --timeout 120 --timeout-method thread > gpurun_out/${TAG}_e3_pytest.log 2>&1 || { echo "stream3 pytest failed"; tail -30 gpurun_out/${TAG}_e3_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_e3_pytest.log
ONLY=encode,split timeout -k 10 200 python scripts/bench_paths.py > gpurun_out/${TAG}_enc_paths.jsonl 2> gpurun_out/${TAG}_enc_paths.err || { echo "encode paths failed"; tail -5 gpurun_out/${TAG}_enc_paths.err; exit 1; }
cat gpurun_out/${TAG}_enc_paths.jsonl
echo "[$(date +%T)] full check"
bash scripts/gpu_check.sh ${TAG}
