"""Summarise rocprofv3 PMC databases (rocpd sqlite): per kernel-name, the mean of each counter over
its dispatches (a dispatch's value summed over the per-SE/XCD rows rocprofv3 stores).

    python scripts/pmc_db.py gpurun_out/pmc/p1/p1_results.db [...] [--match rq_encoder]
"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("dbs", nargs="+")
ap.add_argument("--match", default="")
a = ap.parse_args()
res = collections.defaultdict(lambda: collections.defaultdict(list))
for db in a.dbs:
    c = sqlite3.connect(db)
    per = collections.defaultdict(float)
    names = {}
    for disp, kname, cname, val, vgpr, agpr, dur in c.execute(
            "select dispatch_id, kernel_name, counter_name, value, vgpr_count, accum_vgpr_count, duration "
            "from counters_collection"):
        if a.match and a.match not in kname:
            continue
        per[(disp, cname)] += val
        names[disp] = (kname, vgpr, agpr)
    for (disp, cname), v in per.items():
        res[names[disp]][cname].append(v)
for (kname, vgpr, agpr), cs in res.items():
    print(f"{kname[:110]}  vgpr {vgpr} agpr {agpr}")
    for cname in sorted(cs):
        vals = cs[cname]
        print(f"    {cname:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})")
