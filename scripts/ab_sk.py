"""Device time of the Sinkhorn assignment kernel (gr_rq_encode_sk_f32, csrc/rq_sk.hip) per launch at
training-batch shapes: events around 20 back-to-back launches of one level, eps 0.01, 50 iterations."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
for B, K in [(64, 8), (64, 256), (256, 256), (1024, 8), (4096, 256)]:
    g = torch.Generator(device=dev).manual_seed(0)
    z = torch.randn(B, 32, generator=g, device=dev)
    cb = torch.randn(K, 32, generator=g, device=dev)
    for _ in range(3):
        ops.rq_quantize_sk(z, [cb], [0.01], 50)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        ops.rq_quantize_sk(z, [cb], [0.01], 50)
    b.record()
    torch.cuda.synchronize()
    print(f"B {B:5d} K {K:4d}: {a.elapsed_time(b) / 20 * 1e3:8.1f} us per level", flush=True)
