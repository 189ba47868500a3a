"""A/B timing of the SASRec forward paths (steady state, HIP events): per option setting, the
mean device time of ``model.last_hidden`` (predict's forward) and ``model.forward`` (all positions).

    python scripts/ab_sas.py [--d 128 --n 200 --B 512 --items 1000000] [--opt emb_proj=0,1]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, synth  # noqa: E402

if os.environ.get("GR_DIAG_LIB"):   # diagnostic build (build.py --abl MACRO): results may be wrong
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["GR_DIAG_LIB"])


def timeit(fn, reps=30, spin=0.5):
    import time
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
ap.add_argument("--d", type=int, default=128)
ap.add_argument("--n", type=int, default=200)
ap.add_argument("--B", type=int, default=512)
ap.add_argument("--items", type=int, default=1_000_000)
ap.add_argument("--fused", type=int, default=1)
ap.add_argument("--opt", default="emb_proj=0,1")
a = ap.parse_args()
dev = torch.device("cuda:0")
p = synth.sasrec_params(a.d, a.n, 2, 1, 64, dev)
m = synth.sasrec_model(a.items, p, dev, seed=5)
seqs = synth.sequences(a.B, a.n, a.items, 5000, dev)
_lib.set_option("sas_fused", a.fused)
name, vals = a.opt.split("=")
ref = None
for v in vals.split(","):
    _lib.set_option(name, int(v))
    h = m.last_hidden(seqs)
    f = m.forward(seqs[:64])
    if ref is None:
        ref = (h, f)
    same = (torch.equal(h, ref[0]), torch.equal(f, ref[1]))
    print(f"{name}={v}: last_hidden {timeit(lambda: m.last_hidden(seqs)) * 1e3:8.1f} us   "
          f"forward(all positions, B=64) {timeit(lambda: m.forward(seqs[:64])) * 1e3:8.1f} us   "
          f"bitwise same as first setting: {same}", flush=True)
