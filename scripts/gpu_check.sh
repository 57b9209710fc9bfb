#!/bin/bash
# GPU-box check: parity tests, smoke, bench, rocprof kernel stats.  Each GPU step
# has its own time limit; steps are chained so the first failure ends the run.
#   SKIP_SLOW=1   skip the BASELINE-size tests
#   PROBE_T=1     run the encode segment-timing probe (bench_tools/stream_probe <sc> t) first
#   PMC=1         PMC passes of the encode after the profile
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-run}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
if [ -n "$PROBE_T" ]; then
echo "[$(date +%T)] encode segment timing"
timeout -k 10 120 ./bench_tools/stream_probe 419432 t > gpurun_out/${TAG}_timing.txt 2>&1 || { echo "probe failed rc=$?"; tail -20 gpurun_out/${TAG}_timing.txt; exit 1; }
cat gpurun_out/${TAG}_timing.txt
fi
echo "[$(date +%T)] pytest -m gpu (not slow)"
timeout -k 10 600 $PYT tests -m "gpu and not slow" > gpurun_out/${TAG}_pytest_fast.log 2>&1 || { echo "pytest fast failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest_fast.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_fast.log
if [ -z "$SKIP_SLOW" ]; then
echo "[$(date +%T)] pytest -m 'gpu and slow' (BASELINE sizes)"
timeout -k 10 900 $PYT tests -m "gpu and slow" > gpurun_out/${TAG}_pytest_slow.log 2>&1 || { echo "pytest slow failed rc=$?"; tail -40 gpurun_out/${TAG}_pytest_slow.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest_slow.log
fi
echo "[$(date +%T)] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
echo "[$(date +%T)] bench"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; }
tail -2 gpurun_out/${TAG}_bench.log
echo "[$(date +%T)] rocprofv3 kernel trace"
export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o enc --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-verify --no-host-path --cpu-seconds 0 ) > gpurun_out/${TAG}_rocprof.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/${TAG}_rocprof.log; exit 1; }
find gpurun_out/${TAG}_prof -type f ! -name "*stats*" -delete
find gpurun_out/${TAG}_prof -name "*stats*"
if [ -n "$PMC" ]; then
echo "[$(date +%T)] PMC passes"
bash scripts/prof_pmc.sh ${TAG}_pmc auto 0 || { echo "pmc failed"; exit 1; }
fi
echo "[$(date +%T)] done"
