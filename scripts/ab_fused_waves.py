#!/usr/bin/env python3
"""A/B of the fused d <= 64 SASRec forward: one wave per sequence (sas_fused=1) against two waves
per sequence (sas_fused=3, one 32-token tile per wave) and the batch-size rule (sas_fused=2) over the batch size, at the C3 shape
(d 64, n 50, 2 blocks, 1 head, mlp 64).  Device time per call (HIP events, 30 calls after a 0.5 s
spin-up) of last_hidden (predict's forward: the final block as the H-form tail) and of forward
(every position); outputs are bitwise equal (tests/test_sasrec_gpu.py)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, synth  # noqa: E402


def dev_us(fn, reps=30):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    d, n = int(os.environ.get("D", 64)), int(os.environ.get("N", 50))
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    m = synth.sasrec_model(100_000, p, dev, seed=5)
    for B in (128, 256, 512, 768, 1024, 1536, 2048):
        seqs = synth.sequences(B, n, 100_000, 5000, dev)
        row = []
        for opt in (1, 3, 2):
            _lib.set_option("sas_fused", opt)
            row.append((dev_us(lambda: m.last_hidden(seqs)), dev_us(lambda: m.forward(seqs))))
        _lib.set_option("sas_fused", 2)
        print(f"B {B:5d}: last_hidden 1 wave {row[0][0]:7.1f} us, 2 waves {row[1][0]:7.1f} us, "
              f"auto {row[2][0]:7.1f} us | forward 1 wave {row[0][1]:7.1f} us, 2 waves {row[1][1]:7.1f} us, "
              f"auto {row[2][1]:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
