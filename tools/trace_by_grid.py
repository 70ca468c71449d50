"""Per-dispatch rocprofv3 kernel trace -> average duration per (kernel, grid).

usage: trace_by_grid.py <rocprofv3 -d dir> [name substring]

`--kernel-trace --stats` averages over every launch of one kernel name;
a probe that launches one kernel at several sizes needs the per-dispatch
trace (*kernel_trace.csv) split by grid size instead.  Prints one JSON line
per (kernel, grid): launches, mean / median / min microseconds.
"""
import csv
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
rows = {}
for f in sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)):
    with open(f) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name", "")
            if sub not in name:
                continue
            grid = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
            dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            rows.setdefault((name, grid), []).append(dt)
for (name, grid), ts in sorted(rows.items(), key=lambda kv: (kv[0][0], int(kv[0][1]) if kv[0][1].isdigit() else 0)):
    print(json.dumps({"kernel": name[:140], "grid": grid, "launches": len(ts),
                      "mean_us": round(statistics.mean(ts), 2), "median_us": round(statistics.median(ts), 2),
                      "min_us": round(min(ts), 2)}))
