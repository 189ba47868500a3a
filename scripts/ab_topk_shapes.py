#!/usr/bin/env python3
"""A/B of gr_score_topk_f32's tile size (option topk_half: 16-row half tiles vs 32-row tiles) at
the C5 shapes: the 1M-row single-GPU call (512 users), one 125k-row shard with 512 users (the old
per-rank leg) and with 4096 users (the c5_rank leg: 512 users per rank x 8 ranks).  Device time
per call from HIP events over 50 back-to-back calls after a 0.5 s spin-up; results are bitwise
equal across the options (tests/test_score_topk_gpu.py)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops, synth  # noqa: E402


def dev_ms(fn, reps=50):
    torch.cuda.synchronize()
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
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    d, k = 128, 10
    table = synth.table_rows(torch.arange(1_000_001, device=dev), d, 7, dev)
    g = torch.Generator(device=dev).manual_seed(1)
    for B, rows in ((512, 1_000_001), (512, 125_000), (4096, 125_000), (2048, 250_000)):
        h = torch.randn(B, d, generator=g, device=dev) * 0.3
        shard = table[:rows]
        ts = torch.zeros(B, device=dev)
        res = {}
        for half in (0, 1, 2):
            _lib.set_option("topk_half", half)
            res[half] = dev_ms(lambda: ops.score_topk(h, shard, k, 0, thresholds=ts, mask_col0=True))
        _lib.set_option("topk_half", 2)
        fl = 2 * d * rows * B
        print(f"B {B:5d} rows {rows:8d}: " + "  ".join(
            f"half={hf}: {ms * 1e3:8.1f} us ({fl / (ms * 1e-3) / 1e12 / 157.3:.3f})" for hf, ms in res.items()),
            flush=True)


if __name__ == "__main__":
    main()
