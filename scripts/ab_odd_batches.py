"""Device time of the scoring launches at batch sizes whose user blocks do not divide the resident
workgroups (gr_score_f32 into contiguous [B, N+1] logits, gr_score_count_gt_f32, d 64, 100,001
rows) for several builds (scripts/build_variant.sh tags; "base" = the default build), results
compared bitwise against the first tag."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops  # noqa: E402


def dev_us(fn, reps=20):
    for _ in range(5):
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
base = os.path.dirname(_lib.LIB_PATH)
default = _lib.LIB_PATH
tags = sys.argv[1:] or ["base"]
rows = 100_001
table = torch.randn(rows, 64, generator=g, device=dev)
res = {t: {} for t in tags}
same = {t: True for t in tags}
ref = {}
for rnd in range(2):
    for B in (700, 1000, 1500, 3000):
        h = torch.randn(B, 64, generator=g, device=dev)
        thr = torch.randn(B, generator=g, device=dev)
        out = torch.empty(B, rows, device=dev)
        for t in tags:
            _lib._lib = None
            _lib.LIB_PATH = default if t == "base" else os.path.join(base, f"libgr_amd_{t}.so")
            us_s = dev_us(lambda: ops.score(h, table, out=out))
            us_c = dev_us(lambda: ops.score_count_gt(h, table, thr))
            c = ops.score_count_gt(h, table, thr)
            torch.cuda.synchronize()
            key = (rnd, B)
            if t == tags[0]:
                ref[key] = (out.clone(), c.clone())
            else:
                same[t] &= torch.equal(out, ref[key][0]) and torch.equal(c, ref[key][1])
            res[t].setdefault(B, []).append((us_s, us_c))
for t in tags:
    print(t, "  ".join(f"B {B}: score {min(v)[0]:7.1f} us count {min(x[1] for x in v):7.1f} us" for B, v in res[t].items()),
          f"| equal to {tags[0]}: {same[t]}", flush=True)
