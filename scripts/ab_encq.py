"""A/B of RQVAE.get_indices at the fused encoder shape: rq_encq=1 (one launch: encoder + claimed
quantize phase) against rq_encq=0 (encoder and quantize kernels back to back), same library, same
inputs; device time of 20 graph-captured calls per replay, and whether the IDs are bitwise equal.

    python scripts/ab_encq.py [--n 100000,409600] [--L 3 --K 256] [--reps 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib as L, ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", default="100000,409600")
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
dev = torch.device("cuda:0")


def graph_us(fn, calls=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    for _ in range(30):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * calls) * 1e3


rq = synth.rqvae_model(a.L, a.K, dev)
for n in [int(v) for v in a.n.split(",")]:
    x = synth.items(n, 1000, dev)
    res = {}
    for rep in range(a.reps):
        for encq in (0, 1):
            L.set_option("rq_encq", encq)
            idx = rq.get_indices(x)
            torch.cuda.synchronize()
            if encq not in res:
                res[encq] = idx.clone()
            us = graph_us(lambda: rq.get_indices(x))
            same = torch.equal(idx, res[0]) if 0 in res else None
            print(f"n={n:8d} L={a.L} K={a.K} rq_encq={encq}: {us:8.2f} us/call  "
                  f"({n / us:7.1f} M items/s)  ids equal to rq_encq=0: {same}", flush=True)
    L.set_option("rq_encq", 1)
