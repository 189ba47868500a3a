"""Device time of gr_rq_quantize_f32 at C2 (3 x 256, e 32, 100k items) for the library named by
GR_AMD_LIB (diagnostic variants from scripts/build_variant.sh); 20 calls per replayed graph.

    GR_AMD_LIB=.../libgr_amd_qd1.so python scripts/ab_quant_diag.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops, synth  # noqa: E402


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


dev = torch.device("cuda:0")
m = synth.rqvae_model(3, 256, dev)
for n in (100_000, 409_600):
    x = synth.items(n, 0, dev)
    z = m.encoder(x)
    cbs = m.rq.codebooks()
    us = graph_us(lambda: ops.rq_quantize(z, cbs))
    print(f"{os.path.basename(os.environ.get('GR_AMD_LIB', 'libgr_amd.so')):22s} n={n:7d} quantize {us:7.1f} us")
