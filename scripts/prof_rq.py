"""Run one RQ encode variant repeatedly (for rocprofv3 counter collection).

    python scripts/prof_rq.py --fused 1 --occ 1 [--iters 20 --L 3 --K 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--fused", type=int, default=1)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--items", type=int, default=100_000)
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
a = ap.parse_args()
dev = torch.device("cuda:0")
m = synth.rqvae_model(a.L, a.K, dev)
x = synth.items(a.items, 7, dev)
_lib.set_option("rq_fused", a.fused)
for _ in range(a.iters):
    m.get_indices(x)
torch.cuda.synchronize()
print("done")
