"""Device time of SASRec predict's scoring (gr_score_f32 into the contiguous [B, N+1] logits, C3:
d 64, 100,001 rows) for several builds of the library (scripts/build_variant.sh tags; "base" = the
default build), interleaved in one process: B 2048 (rotated whole lines), 512 and 128 (direct); every tag's
logits are compared bitwise with the first tag's."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops  # noqa: E402


def dev_us(fn, reps=30):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
table = torch.randn(100_001, 64, generator=g, device=dev)
base = os.path.dirname(_lib.LIB_PATH)
default = _lib.LIB_PATH
tags = sys.argv[1:] or ["base"]
res = {t: {} for t in tags}
same = {t: True for t in tags}
for rnd in range(3):
    for B in (2048, 512, 128):
        h = torch.randn(B, 64, generator=g, device=dev)
        out = torch.empty(B, 100_001, device=dev)
        for t in tags:
            _lib._lib = None
            _lib.LIB_PATH = default if t == "base" else os.path.join(base, f"libgr_amd_{t}.so")
            out.fill_(float("nan"))
            res[t].setdefault(B, []).append(dev_us(lambda: ops.score(h, table, out=out)))
            if t == tags[0]:
                ref = out.clone()
            else:
                same[t] &= bool(torch.equal(out, ref))
for t in tags:
    print(t, "  ".join(f"B {B}: {min(v):7.1f} us" for B, v in res[t].items()),
          f"| logits bitwise equal to {tags[0]}: {same[t]}", flush=True)
