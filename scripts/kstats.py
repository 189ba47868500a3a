"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, average / min / max microseconds."""
import csv
import glob
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    print(f"== {d}")
    for r in csv.DictReader(open(f[0])):
        print(f"  {r['Name'][:72]:72s} n={r['Calls']:>5} avg={float(r['AverageNs'])/1e3:9.1f}us "
              f"min={float(r['MinNs'])/1e3:9.1f} max={float(r['MaxNs'])/1e3:9.1f} {float(r['Percentage']):5.1f}%")
