#!/bin/bash
# Planner knob sweep (fold cost x group-merge slack x output duplication) on the
# decode/repair paths, grouped executor.  COMBOS: space-separated fold:slack:dup triples.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-pls}
for combo in ${COMBOS:-24:0:0 24:2:24}; do
  set -- ${combo//:/ }
  CLAY_PLAN_FOLD_COST=$1 CLAY_PLAN_MERGE_SLACK=$2 CLAY_PLAN_DUP=${3:-0} CLAY_EXEC=${EXEC:-grouped} ONLY=${ONLY:-decode,repair} RUNS=${RUNS:-7} PREWARM_MS=100 \
    timeout -k 10 300 python scripts/bench_paths.py > gpurun_out/${TAG}_f$1_s$2_d${3:-0}.jsonl 2> gpurun_out/${TAG}_f$1_s$2_d${3:-0}.err || { echo "sweep $combo failed"; tail -20 gpurun_out/${TAG}_f$1_s$2_d${3:-0}.err; exit 1; }
  python - "$R/gpurun_out/${TAG}_f$1_s$2_d${3:-0}.jsonl" "f$1 s$2 d${3:-0}" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        if "from full" in d["config"]: continue
        print(sys.argv[2], d["config"], d["median_ms"], "ms", d["frac_of_8TBps"], d["path"], d["launches"])
PY
done
