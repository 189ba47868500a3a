#!/usr/bin/env python3
"""A/B of the persistent attention kernel's item order (option attn_group: 1 sequence-grouped, 0
longest-first) inside the C5 forward: bitwise output check and HIP-event time of the layer-wise
forward / last_hidden per order.  ``--only G`` runs one order (for rocprofv3 kernel stats)."""
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
    shapes = [(128, 1, 200, 512), (128, 2, 200, 256), (128, 1, 100, 512), (64, 1, 200, 512)]
    orders = [a.only] if a.only >= 0 else [0, 1, 0, 1]
    out = []
    for d, heads, n, B in shapes:
        p = synth.sasrec_params(d, n, 2, heads, 64, dev)
        m = synth.sasrec_model(2000, p, dev, seed=d + n + heads)
        seqs = synth.sequences(B, n, 2000, 17 + n, dev)
        res = {}
        for g in orders:
            _lib.set_option("attn_group", g)
            f = m.forward(seqs)
            if g in res:
                assert torch.equal(res[g][0], f)
            t_f = dev_ms(lambda: m.forward(seqs))
            t_h = dev_ms(lambda: m.last_hidden(seqs))
            res.setdefault(g, [f, []])[1].append((round(t_f, 4), round(t_h, 4)))
        _lib.set_option("attn_group", 1)
        eq = all(torch.equal(res[g][0], res[orders[0]][0]) for g in res)
        out.append({"shape": [d, heads, n, B], "equal": eq, "ms_forward_last_hidden": {g: res[g][1] for g in res}})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
