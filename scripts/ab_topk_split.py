"""Device time of gr_score_topk_f32 (target threshold counts + top-10) at the c5_rank shape (4,096
users x a 125,000-row shard, d 128), at 3,000 and 2,048 users on the shard and at C5 (512 x 1M rows)
for several builds of the library (scripts/build_variant.sh tags; "base" = the default build),
interleaved in one process, with the results compared bitwise against the first tag."""
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
cases = [(4096, 125_000), (3000, 125_000), (2048, 125_000), (512, 1_000_001)]
data = {}
for B, rows in cases:
    h = torch.randn(B, 128, generator=g, device=dev) * 0.1
    t = torch.randn(rows, 128, generator=g, device=dev) * 0.1
    thr = torch.randn(B, generator=g, device=dev) * 0.1
    data[(B, rows)] = (h, t, thr)
res = {t: {} for t in tags}
ref = {}
same = {t: True for t in tags}
for rnd in range(3):
    for key, (h, t, thr) in data.items():
        for tag in tags:
            _lib._lib = None
            _lib.LIB_PATH = default if tag == "base" else os.path.join(base, f"libgr_amd_{tag}.so")
            out = ops.score_topk(h, t, 10, 0, thresholds=thr, mask_col0=True)
            torch.cuda.synchronize()
            if tag == tags[0]:
                ref[key] = [o.clone() for o in out]
            else:
                same[tag] &= all(torch.equal(a, b) for a, b in zip(out, ref[key]))
            res[tag].setdefault(key, []).append(dev_us(lambda: ops.score_topk(h, t, 10, 0, thresholds=thr,
                                                                            mask_col0=True)))
for tag in tags:
    print(tag, "  ".join(f"B {B} x {rows}: {min(v):8.1f} us" for (B, rows), v in res[tag].items()),
          f"| results equal to {tags[0]}: {same[tag]}", flush=True)
