"""A/B of the fused encoder's weight-image policy at C2 (100k items, 3x256): packed per call (the
default, robust to any weight update) vs RQVAE.freeze_encoder() (packed once per weight version).
HIP-event steady state per get_indices call; IDs must be bitwise equal.

    python scripts/ab_rq_pack.py [--items 100000]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--items", type=int, default=100_000)
ap.add_argument("--reps", type=int, default=100)
a = ap.parse_args()
dev = torch.device("cuda:0")
m = synth.rqvae_model(3, 256, dev)
x = synth.items(a.items, 0, dev)


def timeit(fn, reps, spin=0.5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < spin:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


ref = m.get_indices(x)
for rep in range(3):
    for frozen in (False, True):
        m.freeze_encoder(frozen)
        us = timeit(lambda: m.get_indices(x), a.reps)
        same = torch.equal(m.get_indices(x), ref)
        print(f"frozen={frozen!s:5s} {us:8.1f} us/call  {a.items / us:7.2f} M items/s  ids equal: {same}", flush=True)
