"""Diagnostic 3: dump the C2 codebooks, the latents of rows where the 8-wave quantizer disagrees with
the host, and the kernel outputs, for off-line analysis of the kernel's arithmetic."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops, synth  # noqa: E402

dev = torch.device("cuda:0")
m = synth.rqvae_model(3, 256, dev)
b = m.encode_binding()
n = 1_000_000
x = synth.items(n, 1000, dev)
z = ops.rq_mlp(x, b.ws, b.bs)
idx, best, gap = ops.rq_quantize(z, b.cbs, with_gap=True)
rows = torch.tensor([28219, 43693, 509859, 740332, 322768], device=dev)
alone = torch.stack([ops.rq_quantize(z[r:r + 1].contiguous(), b.cbs)[0] for r in rows.tolist()])
np.savez(os.path.join("gpurun_out", "rq_dump.npz"), cb0=b.cbs[0].cpu().numpy(), cb1=b.cbs[1].cpu().numpy(),
         cb2=b.cbs[2].cpu().numpy(), rows=rows.cpu().numpy(), z=z[rows].cpu().numpy(),
         idx=idx[rows].cpu().numpy(), best=best[rows].cpu().numpy(), gap=gap[rows].cpu().numpy(),
         alone=alone.cpu().numpy(), zblock=z[43693 - 700:43693 + 700].cpu().numpy(),
         idxblock=idx[43693 - 700:43693 + 700].cpu().numpy())
print("dumped", idx[rows].tolist(), alone.tolist())
