"""A/B of the fused score + top-k kernel (gr_score_topk_f32) against its diagnostic ablations and the
other scoring-chain kernels, HIP events on the launch stream.

    python scripts/ab_topk.py            (C5 shape: B 512, 1,000,001 rows, d 128; and C3: 2048 x 100,001 x 64)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops  # noqa: E402


def ms(fn, reps=50):
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.5:   # clock ramp (bench.py spinup)
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


dev = torch.device("cuda:0")
SHAPES = [(512, 1_000_001, 128), (512, 125_000, 128), (2048, 100_001, 64)]
if os.environ.get("AB_SHAPE"):
    SHAPES = [SHAPES[int(os.environ["AB_SHAPE"])]]
for B, rows, d in SHAPES:
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn((B, d), generator=g, device=dev)
    t = torch.randn((rows, d), generator=g, device=dev)
    thr = torch.randn(B, generator=g, device=dev)
    fl = 2.0 * B * rows * d
    res = {}
    res["count_gt"] = ms(lambda: ops.score_count_gt(h, t, thr))
    for smp in (1, 0):
        _lib.set_option("topk_sample", smp)
        res[f"topk sample{smp}"] = ms(lambda: ops.score_topk(h, t, 10, thresholds=thr))
    _lib.set_option("topk_sample", 1)
    for wpc in (1, 2, 3, 4):
        _lib.set_option("topk_wg_per_cu", wpc)
        res[f"topk wg/cu {wpc}"] = ms(lambda: ops.score_topk(h, t, 10, thresholds=thr))
    _lib.set_option("topk_wg_per_cu", 0)
    _lib.set_option("topk_ablate", 1)
    res["topk no-topk"] = ms(lambda: ops.score_topk(h, t, 10, thresholds=thr))
    _lib.set_option("topk_ablate", 0)
    if B * rows * 4 < 3e9:
        out = torch.empty((B, rows), device=dev)
        res["score (logits)"] = ms(lambda: ops.score(h, t, out=out))
    for k, v in res.items():
        print(f"B {B} rows {rows} d {d}  {k:16s} {v * 1e3:9.1f} us  {fl / v / 1e9:7.1f} TF/s "
              f"({fl / v / 1e9 / 157.3 * 100:4.1f} %)", flush=True)
