"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json: HBM bytes per
launch of each gr:: kernel, PER BENCH LEG and per launch shape (grid), so a kernel launched at two
sizes (the C5 exact pass over 1M rows and over one 125k-row shard) is never averaged together.
FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of wide (16 B/lane)
streaming reads, so it is doubled (MI355X_MICROARCH.md §HBM).

    python scripts/pmc_traffic.py --tag T [--merge profiles/traffic.json] \\
        c2=<fetch_dir>,<write_dir> c5=<fetch_dir>,<write_dir> ...  > profiles/traffic.json

Output: {"legs": {leg: {"<kernel>@<grid>": {"launches", "bytes_per_launch", "read_bytes",
"write_bytes"}}}, "source": ...}.  bench.py sums the kernels of one call (``call_traffic``).
"""
import argparse
import collections
import csv
import glob
import json
import re


def per_group(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter and "gr::" in r["Kernel_Name"]:
            name = re.sub(r"^void ", "", r["Kernel_Name"]).split("(")[0].replace("gr::", "").replace(" ", "")
            vals[f"{name}@{int(r['Grid_Size'])}"].append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="")
    ap.add_argument("--merge", default=None, help="existing traffic.json whose other legs are kept")
    ap.add_argument("legs", nargs="+", help="leg=fetch_dir,write_dir")
    a = ap.parse_args()
    out = {"legs": {}}
    if a.merge:
        try:
            out["legs"].update(json.load(open(a.merge)).get("legs", {}))
        except (OSError, ValueError):
            pass
    for spec in a.legs:
        leg, dirs = spec.split("=", 1)
        fd, wd = dirs.split(",")
        fetch, write = per_group(fd, "FETCH_SIZE"), per_group(wd, "WRITE_SIZE")
        rows = {}
        for k in sorted(set(fetch) | set(write)):
            fv, wv = fetch.get(k, []), write.get(k, [])
            fb = 2 * 1024 * (sum(fv) / len(fv) if fv else 0.0)
            wb = 1024 * (sum(wv) / len(wv) if wv else 0.0)
            rows[k] = {"launches": max(len(fv), len(wv)), "bytes_per_launch": fb + wb,
                       "read_bytes": fb, "write_bytes": wb}
        out["legs"][leg] = rows
    out["source"] = f"rocprofv3 --pmc FETCH_SIZE (x2, gfx950) and --pmc WRITE_SIZE in separate passes, {a.tag}"
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
