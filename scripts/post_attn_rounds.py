"""The C5 forward (d 128, n 200, 2 blocks) at several batch sizes, for a kernel trace of
post_attn8_kernel: one 64-token row tile per 8-wave workgroup, two workgroups per CU, so B 512
(1,600 tiles) takes ceil(1600 / 512) = 4 rounds of workgroups for 3.125 rounds of work.  Run under
rocprofv3 --kernel-trace; the per-grid rows of scripts/trace_stats.py give the kernel time per B."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
p = synth.sasrec_params(128, 200, 2, 1, 64, dev)
m = synth.sasrec_model(100_000, p, dev, seed=5)
for B in (384, 448, 480, 512, 544, 576, 640):
    seqs = synth.sequences(B, 200, 100_000, 7 + B, dev)
    for _ in range(20):
        m.last_hidden(seqs)
    torch.cuda.synchronize()
    print("B", B, "done", flush=True)
