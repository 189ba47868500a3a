"""C5 step (forward of 512 users + fused score/top-10 over the 1M catalog) issued sequentially on one
stream vs split into user sub-batches whose forward and scoring alternate across two streams (the
next sub-batch's transformer overlapping the current one's catalog pass)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import ops, synth  # noqa: E402


def ms(fn, reps=20):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        fn()
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


dev = torch.device("cuda:0")
items, n, B, d = 1_000_000, 200, 512, 128
model = synth.sasrec_model(items, synth.sasrec_params(d, n, 2, 1, 64, dev), dev, seed=5)
seqs = synth.sequences(B, n, items, 5000, dev)
table = model.item_emb.weight.detach()
thr = torch.zeros(B, device=dev)
s2 = torch.cuda.Stream(device=dev)


def seq():
    h = model.last_hidden(seqs)
    return ops.score_topk(h, table, 10, thresholds=thr)


def overlapped(P):
    cuts = [B * j // P for j in range(P + 1)]
    main = torch.cuda.current_stream(dev)
    outs = []
    hs = []
    for j in range(P):
        st = main if j % 2 == 0 else s2
        st.wait_stream(main) if j == 0 else None
        with torch.cuda.stream(st):
            h = model.last_hidden(seqs[cuts[j]:cuts[j + 1]])
            outs.append(ops.score_topk(h, table, 10, thresholds=thr[cuts[j]:cuts[j + 1]]))
    main.wait_stream(s2)
    return outs


s2.wait_stream(torch.cuda.current_stream(dev))
ref = seq()
print(f"sequential: {ms(seq) * 1e3:8.3f} ms", flush=True)
for P in (2, 4):
    o = overlapped(P)
    v = torch.cat([x[0] for x in o]); i = torch.cat([x[1] for x in o]); c = torch.cat([x[2] for x in o])
    print(f"2 streams, {P} sub-batches: {ms(lambda: overlapped(P)) * 1e3:8.3f} ms  "
          f"same top-k ids: {torch.equal(i, ref[1])}  counts: {torch.equal(c, ref[2])}", flush=True)
