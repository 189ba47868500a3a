"""Summarise a rocprofv3 --pmc CSV: per (kernel, grid size), mean of each counter over dispatches.

    python scripts/pmc_summary.py <dir-with-run_counter_collection.csv> [kernel-substring]
"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "gr::"
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if filt in r["Kernel_Name"]:
        g = r.get("Grid_Size") or r.get("Grid_Size_X") or "?"
        vals[(r["Kernel_Name"][:80], g)][r["Counter_Name"]].append(float(r["Counter_Value"]))
for (k, g), cs in vals.items():
    print(f"{k}  grid={g}")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} {sum(v) / len(v):16.1f}  (n={len(v)})")
