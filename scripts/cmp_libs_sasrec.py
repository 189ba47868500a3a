#!/usr/bin/env python3
"""Bitwise comparison of the fused SASRec forward between two builds of the library (e.g. the
committed kernel and a rewrite that must keep its fp32 order): each build runs in its own process
(GR_AMD_LIB), writes last_hidden / forward / predict of seeded models to a file, and the parent
compares them.

    python scripts/cmp_libs_sasrec.py lib/libgr_amd_head.so lib/libgr_amd.so [sas_fused values]
"""
import os
import subprocess
import sys

import torch

SHAPES = [  # d, heads, mlp, n, blocks, B
    (64, 1, 64, 50, 2, 300), (64, 1, 64, 64, 2, 33), (32, 1, 64, 20, 2, 40), (32, 1, 32, 40, 3, 17),
    (64, 1, 128, 50, 2, 9), (16, 1, 64, 20, 2, 64), (48, 2, 96, 40, 2, 11), (64, 2, 64, 50, 2, 5),
]


def child(out, opt):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from gr_amd import _lib, synth
    dev = torch.device("cuda:0")
    _lib.set_option("sas_fused", opt)
    res = []
    for d, heads, mlp, n, blocks, B in SHAPES:
        p = synth.sasrec_params(d, n, blocks, heads, mlp, dev)
        m = synth.sasrec_model(500, p, dev, seed=d + n + blocks)
        seqs = synth.sequences(B, n, 500, 11 + n, dev)
        res.append((m.last_hidden(seqs).cpu(), m.forward(seqs).cpu(), m.predict(seqs).cpu()))
    torch.save(res, out)


def main():
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        return
    libs = sys.argv[1:3]
    opts = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1").split(",")]
    runs = []
    for lib, opt in [(libs[0], 1)] + [(libs[1], o) for o in opts]:
        out = f"gpurun_out/cmp_{os.path.basename(lib)}_{opt}.pt"
        env = dict(os.environ, GR_AMD_LIB=os.path.abspath(lib))
        subprocess.run([sys.executable, __file__, "--child", out, str(opt)], env=env, check=True)
        runs.append((lib, opt, torch.load(out, weights_only=True)))
    ok = True
    for lib, opt, res in runs[1:]:
        for shp, a, b in zip(SHAPES, runs[0][2], res):
            same = [torch.equal(x, y) for x, y in zip(a, b)]
            ok &= all(same)
            print(f"{os.path.basename(lib)} sas_fused={opt} {shp}: last_hidden/forward/predict bitwise equal "
                  f"to {os.path.basename(runs[0][0])}: {same}", flush=True)
    print("ALL EQUAL" if ok else "DIFFERENCES FOUND")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
