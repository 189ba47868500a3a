"""Device time of gr_rq_quantize_f32 on short calls (3 x 256, e 32; n = 64, 512, 2048 items) for the
libraries named on the command line (diagnostic variants from scripts/build_variant.sh, the
default build as "base"); graph-replayed, 20 calls per graph after a clock ramp.

    python scripts/ab_quant_small.py base qd1 qd2 ...
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops, synth  # noqa: E402


def graph_us(fn, calls=20, reps=20):
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
    for _ in range(50):   # clock ramp
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * calls) * 1e3


dev = torch.device("cuda:0")
m = synth.rqvae_model(3, 256, dev)
zs = {n: m.encoder(synth.items(n, 0, dev)) for n in (64, 512, 2048)}
cbs = m.rq.codebooks()
base = os.path.dirname(_lib.LIB_PATH)
for tag in sys.argv[1:] or ["base"]:
    path = _lib.LIB_PATH if tag == "base" else os.path.join(base, f"libgr_amd_{tag}.so")
    _lib._lib = None
    _lib.LIB_PATH = path
    row = []
    for n, z in zs.items():
        row.append(f"n={n}: {graph_us(lambda: ops.rq_quantize(z, cbs)):7.2f} us")
    print(f"{tag:6s} " + "  ".join(row), flush=True)
