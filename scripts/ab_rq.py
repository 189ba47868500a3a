"""A/B timing of the RQ encode paths in one process, interleaved rounds (cdna guide §5.4 rule 24).

    python scripts/ab_rq.py [--items 100000] [--rounds 10] [--L 3 --K 256]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gr_amd  # noqa: E402
from gr_amd import _lib, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--items", type=int, default=100_000)
ap.add_argument("--rounds", type=int, default=10)
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
a = ap.parse_args()
dev = torch.device("cuda:0")
m = synth.rqvae_model(a.L, a.K, dev)
x = synth.items(a.items, 7, dev)
variants = {"fused": 1, "layerwise": 0}
flop = 2 * (768 * 256 + 256 * 128 + 128 * 32) + 2 * a.L * a.K * 32
times = {k: [] for k in variants}
ref = None
for rnd in range(a.rounds):
    for name, fused in variants.items():
        _lib.set_option("rq_fused", fused)
        out = m.get_indices(x)
        if ref is None:
            ref = out
        elif name != "layerwise":
            assert torch.equal(out, ref) or (out != ref).any(1).sum().item() < 10
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(a.iters):
            m.get_indices(x)
        e.record()
        torch.cuda.synchronize()
        times[name].append(s.elapsed_time(e) / a.iters)
for name, ts in times.items():
    med = statistics.median(ts)
    print(f"{name:10s} median {med*1e3:8.1f} us  min {min(ts)*1e3:8.1f} us  "
          f"{a.items / (med * 1e-3) / 1e6:7.1f} M items/s  {flop * a.items / (med * 1e-3) / 1e12:6.1f} TFLOP/s")
