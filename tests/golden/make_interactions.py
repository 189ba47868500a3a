"""Container-only: extract the (student_id, class_id) interaction rows of
stu-major/interaction_records.csv (the config-1 data file of BASELINE.json, read as DATA) into
tests/golden/interactions_c1.npz, so the SASRec dataset tests run without /root/reference.

    python tests/golden/make_interactions.py
"""
import csv
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = "/root/reference/stu-major/interaction_records.csv"

with open(SRC, encoding="utf-8-sig", newline="") as f:
    rows = [r for r in csv.DictReader(f)]
keep = [r for r in rows if (r.get("student_id") or "").strip()]
np.savez_compressed(os.path.join(HERE, "interactions_c1.npz"),
                    row_id=np.array([int(r["id"]) for r in keep], np.int64),
                    student_id=np.array([r["student_id"] for r in keep]),
                    class_id=np.array([int(r["class_id"]) for r in keep], np.int64),
                    n_rows_total=np.int64(len(rows)))
print(len(keep), "interactions of", len(rows), "rows")
