#!/bin/bash
# Round 6: breakdown of k_stream_fused2<.., TWO> by probe (libclay_amd_probe.so).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-r06k}
PATS=${PATS:-"0,4,8,12 0,1,4,8 0,1,4,5 8,9,0,4"}
for p in ${PROBES-0 31 34 35 32}; do
  echo "[$(date +%T)] probe $p"
  CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_DECODE_PROBE=$p timeout -k 10 200 python scripts/time_decode.py $PATS > gpurun_out/${TAG}_p$p.txt 2>&1 || { echo "probe $p failed"; tail -5 gpurun_out/${TAG}_p$p.txt; exit 1; }
  grep median gpurun_out/${TAG}_p$p.txt
done
echo "[$(date +%T)] timing probe"
CLAY_AMD_LIB=$R/clay_amd/libclay_amd_probe.so CLAY_DECODE_PROBE=40 timeout -k 10 200 python scripts/time_decode.py $PATS > gpurun_out/${TAG}_p40.txt 2>&1 || { echo "probe 40 failed"; tail -5 gpurun_out/${TAG}_p40.txt; exit 1; }
python - "gpurun_out/${TAG}_p40.txt" <<'PY'
import sys
last = {}
cur = None
for ln in open(sys.argv[1]):
    if "f2-timing" in ln:
        k = "loader" if "loader" in ln else ln.split()[2]  # compute wave w0 / w4
        last[k] = ln.strip()
    if "median" in ln:
        print(ln.strip()); [print("   ", v) for v in last.values()]; last = {}
PY
echo "[$(date +%T)] done"
