#!/usr/bin/env python3
"""pmc_db_summary.py -- per-kernel PMC counters from a rocprofv3 results.db (rocpd SQLite).

Usage: pmc_db_summary.py <results.db> [--json out.json]

Sums every counter over its instances within a dispatch, then averages over the dispatches of
each kernel; also prints the mean dispatch duration.  (rocprofv3 7.x writes results.db by default;
scripts/pmc_summary.py reads the CSV output of older runs.)
"""
import collections
import json
import sqlite3
import sys


def summarize(path):
    db = sqlite3.connect(path)
    cur = db.cursor()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    name_of = {}
    for disp, kname, cname, val, d in cur.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"):
        per[disp][cname] += val
        dur[disp] = d
        name_of[disp] = kname
    out = collections.OrderedDict()
    for disp in sorted(per):
        k = name_of[disp]
        e = out.setdefault(k, {"dispatches": 0, "duration_ns": 0.0, "counters": collections.defaultdict(float)})
        e["dispatches"] += 1
        e["duration_ns"] += dur[disp]
        for c, v in per[disp].items():
            e["counters"][c] += v
    res = {}
    for k, e in out.items():
        n = e["dispatches"]
        res[k] = {"dispatches": n, "mean_duration_ms": e["duration_ns"] / n / 1e6,
                  "per_dispatch": {c: v / n for c, v in sorted(e["counters"].items())}}
    return res


def main():
    res = summarize(sys.argv[1])
    for k, e in res.items():
        cs = "  ".join(f"{c} {v / 1e6:.2f}M" for c, v in e["per_dispatch"].items())
        print(f"{k}: n={e['dispatches']} {e['mean_duration_ms']:.4f} ms  {cs}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
