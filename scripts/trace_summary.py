#!/usr/bin/env python3
"""Kernel-time summary of a rocprofv3 --kernel-trace CSV: mean / median / min / max over the
launches of kernels whose name contains SUBSTR, the first --skip of them dropped (a prewarm).
Usage: trace_summary.py <kernel_trace.csv> <substr> [--skip N]; prints one JSON line."""
import csv
import json
import sys

path, sub = sys.argv[1], sys.argv[2]
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ds = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[skip:])
n = len(ds)
print(json.dumps({"kernel": rows[0]["Kernel_Name"] if rows else sub, "launches": len(rows), "skipped": skip,
                  "counted": n, "mean_ms": round(sum(ds) / n, 4) if n else None,
                  "median_ms": round(ds[n // 2], 4) if n else None, "min_ms": round(ds[0], 4) if n else None,
                  "max_ms": round(ds[-1], 4) if n else None}))
