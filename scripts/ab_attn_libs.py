#!/usr/bin/env python3
"""A/B of the SASRec forward (C5 shapes: the row-tile chain and its attention; C3 / d 16: the fused kernel) between builds
of the library: each build runs in its own process (GR_AMD_LIB), times last_hidden / forward with HIP
events (steady state) and saves the outputs; the parent checks them bitwise against the first build.

    python scripts/ab_attn_libs.py ai-education-generative-recommendation_amd/lib/libgr_amd.so lib/libgr_amd_X.so
"""
import json
import os
import subprocess
import sys

import torch

SHAPES = [  # d, heads, n, B (the last two: the fused d <= 64 forward -- C3, and main.py's d 16)
    (128, 1, 200, 512), (128, 2, 200, 256), (128, 1, 100, 300), (64, 1, 200, 128), (128, 1, 65, 7),
    (64, 1, 50, 2048), (16, 1, 20, 128),
]


def dev_ms(fn, reps=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def child(out):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gr_amd import synth
    dev = torch.device("cuda:0")
    res, times = [], []
    for d, heads, n, B in SHAPES:
        p = synth.sasrec_params(d, n, 2, heads, 64, dev)
        m = synth.sasrec_model(2000, p, dev, seed=d + n + heads)
        seqs = synth.sequences(B, n, 2000, 17 + n, dev)
        res.append((m.last_hidden(seqs).cpu(), m.forward(seqs).cpu()))
        times.append((dev_ms(lambda: m.last_hidden(seqs)), dev_ms(lambda: m.forward(seqs))))
    torch.save(res, out)
    print(json.dumps(times))


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    libs = sys.argv[1:]
    runs = []
    for rep in range(2):
        for lib in libs:
            out = f"/tmp/ab_attn_{os.path.basename(lib)}.pt"
            env = dict(os.environ, GR_AMD_LIB=os.path.abspath(lib))
            p = subprocess.run([sys.executable, __file__, "--child", out], env=env, check=True,
                               capture_output=True, text=True)
            times = json.loads(p.stdout.strip().splitlines()[-1])
            runs.append((lib, times, torch.load(out, weights_only=True)))
    ok = True
    for lib, times, res in runs:
        same = [all(torch.equal(x, y) for x, y in zip(a, b)) for a, b in zip(runs[0][2], res)]
        ok &= all(same)
        print(os.path.basename(lib), " ".join(f"{s}: last_hidden {t[0]:.4f} ms forward {t[1]:.4f} ms"
                                              f" eq={e}" for s, t, e in zip(SHAPES, times, same)), flush=True)
    print("ALL EQUAL" if ok else "DIFFERENCES FOUND")


if __name__ == "__main__":
    main()
