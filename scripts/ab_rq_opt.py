"""Device-time A/B of RQVAE.get_indices under gr_set_option settings (graph-captured, 20 calls per
replay), same inputs; IDs compared bitwise with the first setting.

    python scripts/ab_rq_opt.py --opt rq_fused=0,1 [--n 100000,65536] [--L 3 --K 256]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib as L, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--opt", default="rq_fused=0,1")
ap.add_argument("--n", default="100000")
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--reps", type=int, default=2)
a = ap.parse_args()
dev = torch.device("cuda:0")
name, vals = a.opt.split("=")
vals = [int(v) for v in vals.split(",")]


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
default = L.get_option(name)
for n in [int(v) for v in a.n.split(",")]:
    x = synth.items(n, 1000, dev)
    ref = None
    for rep in range(a.reps):
        for v in vals:
            L.set_option(name, v)
            idx = rq.get_indices(x)
            torch.cuda.synchronize()
            ref = idx.clone() if ref is None else ref
            us = graph_us(lambda: rq.get_indices(x))
            print(f"n={n:8d} L={a.L} K={a.K} {name}={v}: {us:8.2f} us/call ({n / us:7.1f} M items/s)  "
                  f"ids equal to the first setting: {torch.equal(idx, ref)}", flush=True)
L.set_option(name, default)
