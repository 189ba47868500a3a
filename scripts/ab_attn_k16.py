#!/usr/bin/env python3
"""A/B of the hd 64 / 128 attention kernels (option attn_k16: 1 = 32-query tiles over 16-key steps at
two waves per SIMD, 0 = the persistent 32 x 32-step kernel) inside the layer-wise SASRec forward:
HIP-event time of forward / last_hidden per form, and the largest difference between the two
forms' outputs (different fp32 chains; the oracle bound is tests/test_sasrec_gpu.py's).
``--only V`` runs one form (for rocprofv3 kernel statistics)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, synth  # noqa: E402


def dev_ms(fn, reps=30):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", type=int, default=-1)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    shapes = [(128, 1, 200, 512), (128, 2, 200, 256), (128, 1, 100, 512), (64, 1, 200, 512), (128, 1, 65, 7)]
    forms = [a.only] if a.only >= 0 else [0, 1, 0, 1]
    old = _lib.get_option("attn_k16")
    try:
        for d, heads, n, B in shapes:
            p = synth.sasrec_params(d, n, 2, heads, 64, dev)
            m = synth.sasrec_model(2000, p, dev, seed=d + n + heads)
            seqs = synth.sequences(B, n, 2000, 17 + n, dev)
            res = {}
            for f in forms:
                _lib.set_option("attn_k16", f)
                out = m.forward(seqs)
                t = (round(dev_ms(lambda: m.forward(seqs)), 4), round(dev_ms(lambda: m.last_hidden(seqs)), 4))
                res.setdefault(f, [out, []])[1].append(t)
            diff = None
            if 0 in res and 1 in res:
                diff = float((res[0][0] - res[1][0]).abs().max())
            print(json.dumps({"shape": [d, heads, n, B], "max_abs_diff_forms": diff,
                              "ms_forward_last_hidden": {f: res[f][1] for f in res}}), flush=True)
    finally:
        _lib.set_option("attn_k16", old)


if __name__ == "__main__":
    main()
