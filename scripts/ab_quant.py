"""Time gr_rq_quantize_f32 alone (z already encoded) across item counts and levels, HIP events.

    python scripts/ab_quant.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)


def ms(fn, reps=50):
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:   # clock ramp
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for L, K in [(3, 256), (1, 256), (4, 1024)]:
    cbs = [torch.randn((K, 32), generator=g, device=dev) * 0.3 for _ in range(L)]
    for n in (25_000, 50_000, 100_000, 200_000, 400_000):
        z = torch.randn((n, 32), generator=g, device=dev)
        t = ms(lambda: ops.rq_quantize(z, cbs))
        fl = 2.0 * n * L * K * 32
        print(f"L={L} K={K} n={n:7d}: {t * 1e3:8.1f} us  {fl / t / 1e9:6.1f} TF/s  {n / t / 1e3:8.1f} M items/s", flush=True)
