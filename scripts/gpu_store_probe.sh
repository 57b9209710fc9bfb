#!/bin/bash
# write-path investigation: store-kernel sweep + the runtime fill kernel's
# launch shape from a kernel trace of hipMemsetAsync
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" && mkdir -p gpurun_out
TAG=${1:-store}
timeout -k 10 300 ./bench_tools/store_probe ${PROBE_MODE:-all} > gpurun_out/${TAG}_store_probe.txt 2>&1 || { echo "store_probe failed"; tail -5 gpurun_out/${TAG}_store_probe.txt; exit 1; }
cat gpurun_out/${TAG}_store_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_memset_trace" -o memset --output-format csv -- "$R/bench_tools/store_probe" memset > "$R/gpurun_out/${TAG}_memset_trace.log" 2>&1 || { echo "trace failed"; tail -20 "$R/gpurun_out/${TAG}_memset_trace.log"; exit 1; }
f=$(find "$R/gpurun_out/${TAG}_memset_trace" -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'EOF'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
seen = collections.OrderedDict()
for r in rows:
    key = (r.get("Kernel_Name"), r.get("Grid_Size_X", r.get("Grid_Size")), r.get("Workgroup_Size_X", r.get("Workgroup_Size")),
           r.get("VGPR_Count", r.get("Arch_VGPR_Count")), r.get("SGPR_Count"), r.get("LDS_Block_Size", r.get("Lds_Size")))
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    seen.setdefault(key, []).append(d)
for k, v in seen.items():
    print(k, "n=%d" % len(v), "median_us=%.1f" % (sorted(v)[len(v) // 2] / 1e3))
print(list(rows[0].keys()))
EOF
