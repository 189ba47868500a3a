"""gr_linear_f32 at 4 vs 8 waves per workgroup (option lin_w8) over the layer shapes the paths use:
steady-state HIP-event time and bitwise equality of the two settings."""
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


dev = torch.device("cuda:0")
for M, K, N, act, res in [(102400, 128, 384, "none", False), (102400, 128, 256, "none", False),
                          (102400, 128, 128, "none", True), (102400, 128, 64, "relu", False),
                          (102400, 64, 128, "none", True), (100000, 768, 256, "relu", False),
                          (100000, 256, 128, "relu", False), (100000, 128, 32, "none", False)]:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, generator=g, device=dev)
    w = torch.randn(N, K, generator=g, device=dev) * 0.1
    b = torch.randn(N, generator=g, device=dev)
    r = torch.randn(M, N, generator=g, device=dev) if res else None
    fl = 2.0 * M * N * K
    outs, ts = [], []
    for v in (0, 1):
        _lib.set_option("lin_w8", v)
        outs.append(ops.linear(x, w, b, act=act, residual=r))
        ts.append(ms(lambda: ops.linear(x, w, b, act=act, residual=r)))
    print(f"M {M} K {K} N {N} {act}{' +res' if res else ''}: 4 waves {ts[0] * 1e3:7.1f} us "
          f"({fl / ts[0] / 1e9 / 157.3 * 100:4.1f} %)  8 waves {ts[1] * 1e3:7.1f} us "
          f"({fl / ts[1] / 1e9 / 157.3 * 100:4.1f} %)  bitwise equal: {torch.equal(outs[0], outs[1])}", flush=True)
_lib.set_option("lin_w8", 1)
