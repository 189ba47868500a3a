"""One gr_set_option switch on gr_score_topk_f32 at the C5 shard and full C5 shapes (and C3's d 64):
steady-state HIP-event time and bitwise equality of (values, ids, counts) across the settings.

    python scripts/ab_topk_opt.py [--opt topk_half=0,1,2]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops  # noqa: E402


def ms(fn, reps=50):
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


ap = argparse.ArgumentParser()
ap.add_argument("--opt", default="tile_w8=0,1")
a = ap.parse_args()
name, vals = a.opt.split("=")
dev = torch.device("cuda:0")
for B, rows, d in [(512, 125_000, 128), (512, 1_000_001, 128), (2048, 100_001, 64)]:
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn((B, d), generator=g, device=dev)
    t = torch.randn((rows, d), generator=g, device=dev)
    thr = torch.randn(B, generator=g, device=dev)
    fl = 2.0 * B * rows * d
    ref = None
    for v in vals.split(","):
        _lib.set_option(name, int(v))
        out = ops.score_topk(h, t, 10, thresholds=thr)
        ref = out if ref is None else ref
        same = all(torch.equal(x, y) for x, y in zip(out, ref))
        tm = ms(lambda: ops.score_topk(h, t, 10, thresholds=thr))
        print(f"B {B} rows {rows} d {d} {name}={v}: {tm * 1e3:8.1f} us ({fl / tm / 1e9 / 157.3 * 100:4.1f} %)  "
              f"bitwise same as first: {same}", flush=True)
