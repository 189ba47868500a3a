import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib, ops
dev = torch.device("cuda:0")
for B, rows, d in [(300, 100001, 64), (256, 100001, 64), (2048, 100001, 64), (512, 20000, 128)]:
    g = torch.Generator().manual_seed(B + rows)
    h = torch.randn(B, d, generator=g).to(dev)
    t = torch.randn(rows, d, generator=g).to(dev)
    _lib.set_option("score_flags", 0)
    ref = ops.score(h, t)
    _lib.set_option("score_flags", 1)
    _lib.set_option("score_impl", int(os.environ.get("DBG_IMPL", "0")))
    for rep in range(3):
        y = ops.score(h, t)
        bad = (y != ref).nonzero()
        print(B, rows, d, "rep", rep, "mismatches", bad.shape[0], flush=True)
        if bad.shape[0]:
            r_, c_ = bad[:, 0], bad[:, 1]
            print("  rows", r_.min().item(), r_.max().item(), "unique rows", r_.unique().numel(),
                  "cols", c_.min().item(), c_.max().item(), "cols mod 32 hist", torch.bincount(c_ % 32, minlength=32).tolist()[:8], flush=True)
            print("  sample", bad[:5].tolist(), y[bad[0,0], bad[0,1]].item(), ref[bad[0,0], bad[0,1]].item(), flush=True)
