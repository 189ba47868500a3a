"""Device time of rq_quantize_kernel vs n, for a rocprofv3 kernel trace (grid size tells the n
apart): gr_rq_quantize_f32 at C2 codebooks (3 x 256, e 32) on n = 3.2k ... 409.6k items.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 scripts/quant_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops, synth  # noqa: E402

dev = torch.device("cuda:0")
m = synth.rqvae_model(3, 256, dev)
b = m.encode_binding()
for n in (3200, 12800, 25600, 51200, 100_000, 204_800, 409_600):
    x = synth.items(n, 1000, dev)
    z = ops.rq_mlp(x, b.ws, b.bs)
    for _ in range(30):
        ops.rq_quantize(z, b.cbs)
    torch.cuda.synchronize()
    print("n", n, "done", flush=True)
