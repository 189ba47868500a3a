"""Per-launch-shape kernel statistics from a rocprofv3 ``--kernel-trace`` CSV.

rocprofv3's ``kernel_stats.csv`` averages every launch of a kernel name together, so one name
launched at two sizes (the C2 and C4 encoder, a LayerNorm over all tokens and over the last ones)
gives an average that matches neither.  This groups launches by (name, grid, workgroup) and, with
``--leg``, tags the rows, so each bench leg's roofline can be recomputed from the committed CSV.

    python scripts/trace_stats.py <run_kernel_trace.csv> [--leg c2] [--top 25] > stats.csv
"""
import argparse
import csv
import statistics
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--leg", default="")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    groups = {}
    for r in csv.DictReader(open(a.trace)):
        if r.get("Kind", "KERNEL_DISPATCH") != "KERNEL_DISPATCH":
            continue
        key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]),
               int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"]))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    total = sum(sum(v) for v in groups.values()) or 1.0
    # the library's kernels, plus anything else above 0.5 % of the leg (torch set-up kernels of the
    # synthetic inputs are noise)
    rows = [kv for kv in sorted(groups.items(), key=lambda kv: -sum(kv[1]))
            if "gr::" in kv[0][0] or sum(kv[1]) >= 0.005 * total][:a.top]
    w = csv.writer(sys.stdout)
    w.writerow(["leg", "kernel", "grid_threads", "workgroup", "calls", "mean_us", "median_us", "min_us",
                "max_us", "total_ms", "pct_of_leg"])
    for (name, grid, wg), ts in rows:
        w.writerow([a.leg, name, grid, wg, len(ts), f"{statistics.fmean(ts):.2f}", f"{statistics.median(ts):.2f}",
                    f"{min(ts):.2f}", f"{max(ts):.2f}", f"{sum(ts) / 1e3:.3f}", f"{100 * sum(ts) / total:.1f}"])


if __name__ == "__main__":
    main()
