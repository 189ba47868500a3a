#!/usr/bin/env python3
"""Device time of RQVAE.get_indices per call at short call sizes (the reference's batch of 64,
RQ-VAE/infer.py:84-95), C2 model (768 -> 256 -> 128 -> 32, 3 x 256 codes): HIP events over 50
back-to-back calls after a 0.5 s spin-up, and per call of 20 calls captured as one graph.  Run once per library build (GR_AMD_LIB) to compare the
short-call kernels (rq_small.hip) with the long-call kernels on the same sizes."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import synth  # noqa: E402


def dev_us(fn, reps=50):
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
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda:0")
    m = synth.rqvae_model(3, 256, dev)
    x = synth.items(4096, 1000, dev)
    tag = os.path.basename(os.environ.get("GR_AMD_LIB", "libgr_amd.so"))
    for n in [int(v) for v in os.environ.get("NS", "16,32,64,128,192,256,512,1024,2048,4096").split(",")]:
        xs = x[:n].contiguous()
        eager = dev_us(lambda: m.get_indices(xs))
        # the same calls captured as one graph (20 calls per replay): device time without the host's
        # per-call Python / launch cost, which bounds the eager loop at these sizes
        m.get_indices(xs)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr):
            for _ in range(20):
                m.get_indices(xs)
        graph = dev_us(lambda: gr.replay(), reps=10) / 20
        print(f"{tag}: get_indices(x[{n:4d}]) {eager:7.1f} us per call back to back, {graph:7.1f} us per call "
              f"in a graph", flush=True)


if __name__ == "__main__":
    main()
