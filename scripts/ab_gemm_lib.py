"""The C5 block-0 in-projection GEMM shape ([102400 x 128] . [384 x 128]^T + b, fp32) on the
library GEMM (torch -> hipBLASLt / rocBLAS) against gr_linear_f32, steady-state HIP events."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops  # noqa: E402


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
torch.backends.cuda.matmul.allow_tf32 = False
for M, K, N in [(102400, 128, 384), (102400, 128, 256), (102400, 128, 128), (100000, 768, 256)]:
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, K, generator=g, device=dev)
    w = torch.randn(N, K, generator=g, device=dev) * 0.1
    b = torch.randn(N, generator=g, device=dev)
    fl = 2.0 * M * N * K
    t_lib = ms(lambda: torch.nn.functional.linear(x, w, b))
    t_gr = ms(lambda: ops.linear(x, w, b))
    d = (torch.nn.functional.linear(x, w, b) - ops.linear(x, w, b)).abs().max().item()
    print(f"M {M} K {K} N {N}: torch/library {t_lib * 1e3:7.1f} us ({fl / t_lib / 1e9 / 157.3 * 100:4.1f} %)  "
          f"gr_linear {t_gr * 1e3:7.1f} us ({fl / t_gr / 1e9 / 157.3 * 100:4.1f} %)  max |diff| {d:.2e}", flush=True)
