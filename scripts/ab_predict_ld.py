"""A/B of SASRec.predict's logits layout at C3 (d 64, n 50, 100k items): the row-padded buffer
(rows 128-B aligned, ld = roundup(N+1, 32)) against a contiguous [B, N+1] tensor (ld = N+1), HIP-event
steady state per call, and whether the logits are bitwise equal.

    python scripts/ab_predict_ld.py [--B 2048,128]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", default="2048,128")
ap.add_argument("--items", type=int, default=100_000)
ap.add_argument("--impls", default="2,3", help="score_impl values to time (gr_amd.h)")
a = ap.parse_args()
dev = torch.device("cuda:0")
p = synth.sasrec_params(64, 50, 2, 1, 64, dev)
m = synth.sasrec_model(a.items, p, dev)
b = ops.SasrecBinding(m)


def timeit(fn, reps=50, spin=0.5):
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


for B in [int(v) for v in a.B.split(",")]:
    seqs = synth.sequences(B, 50, a.items, 5, dev)
    pad = ops.logits_buffer(B, a.items + 1, dev)
    cont = torch.empty((B, a.items + 1), dtype=torch.float32, device=dev)
    ops.sasrec_predict(b, seqs, out=pad)
    ops.sasrec_predict(b, seqs, out=cont)
    torch.cuda.synchronize()
    same = torch.equal(pad, cont)
    from gr_amd import _lib
    ref = pad.clone()
    for rep in range(2):
        for impl in [int(v) for v in a.impls.split(",")]:
            _lib.set_option("score_impl", impl)
            for name, out in (("padded ld", pad), ("contiguous", cont)):
                out.fill_(float("nan"))
                us = timeit(lambda: ops.sasrec_predict(b, seqs, out=out))
                eq = torch.equal(out, ref)
                print(f"B={B:5d} score_impl={impl} {name:10s} ld={out.stride(0):6d}: {us:8.1f} us/call "
                      f"({B / us:6.3f} M seqs/s)  bitwise equal to padded: {eq}", flush=True)
    _lib.set_option("score_impl", 2)
