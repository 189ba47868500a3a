"""Run SASRec predict (config C3 shapes) repeatedly, for rocprofv3 counter collection.

    python scripts/prof_sas.py [--fused 1 --iters 10 --B 2048 --d 64 --n 50 --items 100000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fused", type=int, default=1)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--B", type=int, default=2048)
ap.add_argument("--d", type=int, default=64)
ap.add_argument("--n", type=int, default=50)
ap.add_argument("--items", type=int, default=100_000)
ap.add_argument("--forward-only", type=int, default=0, help="1: last_hidden only (no scoring)")
a = ap.parse_args()
dev = torch.device("cuda:0")
p = synth.sasrec_params(a.d, a.n, 2, 1, 64, dev)
m = synth.sasrec_model(a.items, p, dev)
seqs = synth.sequences(a.B, a.n, a.items, 5, dev)
out = None if a.forward_only else torch.empty((a.B, a.items + 1), dtype=torch.float32, device=dev)
_lib.set_option("sas_fused", a.fused)
b = ops.SasrecBinding(m)
for _ in range(a.iters):
    if a.forward_only:
        m.last_hidden(seqs)
    else:
        ops.sasrec_predict(b, seqs, out=out)
torch.cuda.synchronize()
print("done")
