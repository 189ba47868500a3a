"""Derived per-kernel metrics from scripts/pmc_sas.sh summaries (p1.txt .. p3.txt of one tag):
MFMA-pipe busy fraction = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
(SQ_VALU_MFMA_BUSY_CYCLES counts 64 cycles per v_mfma_f32_32x32x2_f32), VALU and LDS instructions
per MFMA, LDS bank-conflict cycles per LDS-array cycle, and the wave-cycle split (quad-cycles:
parked in s_waitcnt / barrier, issue-stalled, issuing).

    python scripts/pmc_table.py gpurun_out/r03c_pmc [--all]
"""
import argparse
import collections
import os

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("--all", action="store_true", help="include non-gr:: kernels")
a = ap.parse_args()
res = collections.defaultdict(dict)
for f in sorted(os.listdir(a.dir)):
    if not (f.startswith("p") and f.endswith(".txt")):
        continue
    cur = None
    for line in open(os.path.join(a.dir, f)):
        if not line.startswith("    "):
            cur = line.split("  vgpr")[0].strip()
            res[cur]["vgpr"] = line.split("vgpr")[-1].strip() if "vgpr" in line else ""
        elif cur:
            k, v = line.split()[:2]
            res[cur][k] = float(v)
print(f"{'kernel':58s} {'MFMA busy':>9s} {'VALU/MFMA':>9s} {'LDS/MFMA':>8s} {'LDS conf':>8s} "
      f"{'wait':>6s} {'stall':>6s} {'issue':>6s}  vgpr/agpr")
for k, d in res.items():
    if not a.all and "gr::" not in k:
        continue
    grbm = d.get("GRBM_GUI_ACTIVE", 0) / 8 * 1024
    mf = d.get("SQ_INSTS_MFMA", 0)
    busy = d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / grbm if grbm else 0
    wc = d.get("SQ_WAVE_CYCLES", 0) or 1
    name = k.replace("void ", "").replace("gr::", "")
    name = name[:name.find("(")] if "(" in name else name
    print(f"{name[:58]:58s} {busy:9.3f} {d.get('SQ_INSTS_VALU', 0) / mf if mf else 0:9.2f} "
          f"{d.get('SQ_INSTS_LDS', 0) / mf if mf else 0:8.2f} "
          f"{d.get('SQ_LDS_BANK_CONFLICT', 0) / (d.get('SQ_LDS_IDX_ACTIVE', 0) or 1):8.3f} "
          f"{d.get('SQ_WAIT_ANY', 0) / wc:6.2f} {d.get('SQ_WAIT_INST_ANY', 0) / wc:6.2f} "
          f"{d.get('SQ_ACTIVE_INST_ANY', 0) / wc:6.2f}  {d.get('vgpr', '')}")
