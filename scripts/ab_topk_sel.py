"""Select-kernel ablations of the tile design (diagnostic option topk_sel_abl; results are wrong
under an ablation): total gr_score_topk_f32 time at the C5 shard and full C5 shapes."""
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
for B, rows, d in [(512, 125_000, 128), (512, 1_000_001, 128)]:
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn((B, d), generator=g, device=dev)
    t = torch.randn((rows, d), generator=g, device=dev)
    thr = torch.randn(B, generator=g, device=dev)
    for abl in (0, 1, 2, 4, 7):
        _lib.set_option("topk_sel_abl", abl)
        print(f"B {B} rows {rows} abl {abl}: {ms(lambda: ops.score_topk(h, t, 10, thresholds=thr)) * 1e3:8.1f} us", flush=True)
    _lib.set_option("topk_sel_abl", 0)
