#!/bin/bash
# Sweep of the host-streaming pipeline defaults (piece MiB, streams) on the host-buffer API.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
for cfg in "128 2" "128 3" "64 3" "256 2" "32 4"; do
  set -- $cfg
  CLAY_HOST_PIECE_MB=$1 CLAY_HOST_STREAMS=$2 REPS=3 timeout -k 10 200 python scripts/bench_host.py > gpurun_out/sweep_host_$1_$2.jsonl 2>/dev/null || exit 1
done
python3 - <<'PY'
import glob, json
for f in sorted(glob.glob("gpurun_out/sweep_host_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        if d["pinned"]:
            print(f.split("sweep_host_")[1][:-6], d["op"][:24], d["ms"], d["GiBps"])
PY
