"""Device-time A/B of a gr_set_option switch on gr_rq_quantize_f32 (C2 codebooks 3 x 256, e 32 by
default): 20 calls captured in one graph and replayed, so the host's per-call cost (~40-80 us of
Python + ctypes, which bounded scripts/ab_opt.py's quantize numbers) is off the clock.

    python scripts/ab_quant.py --opt rq_fused=0,1 [--L 3 --K 256] [--n 3200,25600,100000]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops, synth  # noqa: E402


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
    for _ in range(20):   # clock ramp
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * calls) * 1e3


ap = argparse.ArgumentParser()
ap.add_argument("--opt", default="rq_fused=0,1")
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--n", default="3200,25600,51200,100000,409600")
ap.add_argument("--second", action="store_true", help="also return best/second (certified path)")
a = ap.parse_args()
dev = torch.device("cuda:0")
m = synth.rqvae_model(a.L, a.K, dev)
b = m.encode_binding()
name, vals = a.opt.split("=")
for n in [int(v) for v in a.n.split(",")]:
    x = synth.items(n, 1000, dev)
    z = ops.rq_mlp(x, b.ws, b.bs)
    ref = None
    for v in vals.split(","):
        _lib.set_option(name, int(v))
        fn = lambda: ops.rq_quantize(z, b.cbs)   # noqa: E731
        out = fn()
        torch.cuda.synchronize()
        ref = out if ref is None else ref
        t = graph_us(fn)
        print(f"quant L={a.L} K={a.K} n={n} {name}={v}: {t:8.2f} us/call  same as first: {torch.equal(out, ref)}",
              flush=True)
    _lib.set_option(name, int(vals.split(",")[0]))
