#!/usr/bin/env python3
"""A/B: one rank's C5 step (the c5_rank leg: forward of 512 users, target logits + fused rank /
top-10 of 4096 users on a 125k-row shard) issued back to back on one stream, against the same steps
with each step's transformer forward on a second stream so that it runs beside the previous step's
scoring (independent user batches of an evaluation loop; every step still does all of its work).
Device time per step from HIP events around 10 steps after a spin-up."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import dist as D, ops, synth  # noqa: E402

dev = torch.device("cuda:0")
W, items, d, n, k = 8, 1_000_000, 128, 200, 10
B = 512 * W
p = synth.sasrec_params(d, n, 2, 1, 64, dev)
seqs = synth.sequences(B, n, items, 5000, dev)
tg = torch.randint(1, items + 1, (B,), generator=torch.Generator(device=dev).manual_seed(6), device=dev)
lo, hi = D.shard_range(items + 1, 0, W)
shard = synth.table_rows(torch.arange(lo, hi, device=dev), d, 7, dev)
model, lseqs = synth.sasrec_rank_model(items, p, seqs[:512], dev, seed=5)
h = torch.cat([model.last_hidden(lseqs)] * W)
own = (tg >= lo) & (tg < hi)
loc = torch.where(own, tg - lo, torch.zeros_like(tg))


def score():
    ts = torch.where(own, ops.score_pairs(h, shard, loc, mask_col0=True), torch.zeros(B, device=dev))
    return ops.score_topk(h, shard, k, lo, thresholds=ts, mask_col0=True)


side = torch.cuda.Stream()


def seq_steps(m):
    for _ in range(m):
        model.last_hidden(lseqs)
        score()


def overlap_steps(m):
    main = torch.cuda.current_stream()
    side.wait_stream(main)              # the batches' inputs are ready
    for _ in range(m):
        with torch.cuda.stream(side):   # step s+1's forward runs while step s is scored
            model.last_hidden(lseqs)
        done = torch.cuda.Event()
        done.record(side)
        main.wait_event(done)           # step s's scoring reads step s's forward output
        score()
    main.wait_stream(side)


def timed(fn, m=10):
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        fn(2)
        torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn(m)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / m


for rnd in range(2):
    a = timed(seq_steps)
    b = timed(overlap_steps)
    print(f"round {rnd}: sequential {a:.3f} ms/step, forward on a side stream {b:.3f} ms/step", flush=True)
