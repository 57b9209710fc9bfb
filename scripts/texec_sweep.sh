#!/bin/bash
# Tile-executor knob sweep (waves per workgroup x LDS budget) on the decode/repair paths.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-txs}
# COMBOS: space-separated waves:lds_kb pairs
for combo in ${COMBOS:-16:160 8:160 16:80 8:80 4:80}; do
  set -- ${combo/:/ }
  CLAY_PLAN_DEBUG=${DBG:-} CLAY_TEXEC_BIG=1 CLAY_TEXEC_WAVES=$1 CLAY_TEXEC_LDS_KB=$2 CLAY_EXEC=tile ONLY=${ONLY:-decode,repair} RUNS=${RUNS:-5} PREWARM_MS=100 \
    timeout -k 10 300 python scripts/bench_paths.py > gpurun_out/${TAG}_w$1_l$2.jsonl 2> gpurun_out/${TAG}_w$1_l$2.err || { echo "sweep $combo failed"; tail -20 gpurun_out/${TAG}_w$1_l$2.err; exit 1; }
  python - "$R/gpurun_out/${TAG}_w$1_l$2.jsonl" "w$1 l$2" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[2], d["config"], d["median_ms"], "ms", d["frac_of_8TBps"], d["path"], d["launches"])
PY
done
