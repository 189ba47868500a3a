"""Diagnostic: ops.RqTrainGraph replayed back to back (sync=False) against replays with a device
synchronisation after each step (sync=True), from the same initial state, dropout 0: the final
parameters must be bitwise equal if no captured node depends on host-side ordering (the memset
hazard of SasTrainGraph.replay).  Also times both."""
import copy
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from gr_amd import ops  # noqa: E402
from test_rq_train_gpu import _model, _opt, _batches  # noqa: E402

dev = torch.device("cuda:0")
base = _model(dev, 0.0, False)
x = _batches(dev, 1)[0]
res = {}
for sync in (True, False):
    m = copy.deepcopy(base)
    opt, sch = _opt(m, dev, warm=0, total=100000, fused=True)   # lr = 1e-3 from the first step
    step = ops.RqTrainGraph(m, opt, x.clone(), sync=sync)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(300):
        step.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 300 * 1e3
    res[sync] = [p.detach().clone() for p in m.parameters()]
    print(f"sync={sync}: {dt:.3f} ms per replay, loss {step.out[0].item():.6f}", flush=True)
same = all(torch.equal(a, b) for a, b in zip(res[True], res[False]))
print("final parameters bitwise equal:", same, flush=True)
