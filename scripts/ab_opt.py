"""A/B timing of one gr_set_option switch on the RQ encode (C2 / C4 shapes) or the C3 predict:
steady-state mean device time per call (HIP events) and bitwise equality of the outputs.

    python scripts/ab_opt.py --what rq --opt rq_resident=0,1 [--L 3 --K 256 --n 100000]
    python scripts/ab_opt.py --what quant --opt rq_resident=0,1
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops, synth  # noqa: E402


def timeit(fn, reps=50, spin=0.5):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < spin:
        fn()
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


ap = argparse.ArgumentParser()
ap.add_argument("--what", default="rq", choices=["rq", "quant", "score", "predict"])
ap.add_argument("--opt", default="rq_resident=0,1")
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--n", type=int, default=100_000)
a = ap.parse_args()
dev = torch.device("cuda:0")
if a.what in ("rq", "quant"):
    m = synth.rqvae_model(a.L, a.K, dev)
    x = synth.items(a.n, 1000, dev)
    b = m.encode_binding()
    z = ops.rq_mlp(x, b.ws, b.bs)
    fn = (lambda: m.get_indices(x)) if a.what == "rq" else (lambda: ops.rq_quantize(z, b.cbs))
else:   # C3 shapes: 2048 users, d 64, 100k items (--n = users)
    sm = synth.sasrec_model(100_000, synth.sasrec_params(64, 50, 2, 1, 64, dev), dev)
    seqs = synth.sequences(a.n if a.n != 100_000 else 2048, 50, 100_000, 2000, dev)
    hh = sm.last_hidden(seqs)
    tab = sm.item_emb.weight.detach()
    outb = ops.logits_buffer(hh.shape[0], tab.shape[0], dev)
    fn = (lambda: ops.score(hh, tab, out=outb)) if a.what == "score" else (lambda: sm.predict(seqs))
name, vals = a.opt.split("=")
ref = None
for v in vals.split(","):
    _lib.set_option(name, int(v))
    out = fn()
    ref = out if ref is None else ref
    t = timeit(fn)
    print(f"{a.what} L={a.L} K={a.K} n={a.n} {name}={v}: {t * 1e3:8.1f} us  "
          f"bitwise same as first: {torch.equal(out, ref)}", flush=True)
