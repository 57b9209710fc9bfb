#!/usr/bin/env python3
"""Summarise scripts/prof_pmc.sh output: per counter, the mean over the encode kernel's
launches (first launch dropped as warm-up).  Usage: pmc_summary.py gpurun_out/<tag> [kernel-substr]
Prints JSON; with --hbm also the per-launch HBM bytes (FETCH_SIZE x2 per the gfx950
correction in MI355X_MICROARCH.md, WRITE_SIZE as is; both reported in KB)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1]
ksub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else "encode"
vals = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(d, "*", "p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if ksub not in r["Kernel_Name"]:
            continue
        vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
out = {}
for name, per in sorted(vals.items()):
    ids = sorted(per)
    use = ids[1:] if len(ids) > 1 else ids
    out[name] = sum(per[i] for i in use) / len(use)
if "FETCH_SIZE" in out and "WRITE_SIZE" in out:
    out["hbm_bytes_per_launch"] = (2 * out["FETCH_SIZE"] + out["WRITE_SIZE"]) * 1024
print(json.dumps(out, indent=1))
