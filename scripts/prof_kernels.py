"""A short, fixed workload for rocprofv3 PMC passes: a few calls of the C5 forward
(model.last_hidden, d 128, n 200, B 512), one C5 catalog shard's score_topk (shard) and/or the C2
encode (get_indices, 100k items).

    rocprofv3 --pmc ... -d OUT -- python3 scripts/prof_kernels.py --what c5fwd,c2 --calls 5
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--what", default="c5fwd,c2")
ap.add_argument("--calls", type=int, default=5)
ap.add_argument("--opt", default="", help="gr_set_option settings, e.g. lin_wres=0,emb_proj=0")
a = ap.parse_args()
if os.environ.get("GR_DIAG_LIB"):   # diagnostic build (build.py --abl MACRO): results may be wrong
    from gr_amd import _lib
    _lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), os.environ["GR_DIAG_LIB"])
if a.opt:
    from gr_amd import _lib
    for kv in a.opt.split(","):
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
dev = torch.device("cuda:0")
what = a.what.split(",")
if "c5fwd" in what:
    seqs = synth.sequences(512, 200, 1_000_000, 5000, dev)
    m, ls = synth.sasrec_rank_model(1_000_000, synth.sasrec_params(128, 200, 2, 1, 64, dev), seqs, dev, seed=5)
    for _ in range(a.calls):
        m.last_hidden(ls)
    torch.cuda.synchronize()
if "shard" in what:   # one C5 catalog shard (125,000 rows) against 512 users: gr_score_topk_f32
    from gr_amd import ops
    h = torch.randn(512, 128, device=dev)
    shard = torch.randn(125_000, 128, device=dev)
    ts = torch.zeros(512, device=dev)
    for _ in range(a.calls):
        ops.score_topk(h, shard, 10, 0, thresholds=ts, mask_col0=True)
    torch.cuda.synchronize()
if "rankshard" in what:   # the c5_rank leg's scoring: 4096 users x one 125,000-row shard
    from gr_amd import ops
    h = torch.randn(4096, 128, device=dev) * 0.3
    shard = synth.table_rows(torch.arange(125_000, device=dev), 128, 7, dev)
    ts = torch.zeros(4096, device=dev)
    for _ in range(a.calls):
        ops.score_topk(h, shard, 10, 0, thresholds=ts, mask_col0=True)
    torch.cuda.synchronize()
if "c2" in what:
    rq = synth.rqvae_model(3, 256, dev)
    x = synth.items(100_000, 1000, dev)
    for _ in range(a.calls):
        rq.get_indices(x)
    torch.cuda.synchronize()
if "rq64" in what:   # the reference's call pattern: get_indices(x[64]) (RQ-VAE/infer.py:84-95)
    rq = synth.rqvae_model(3, 256, dev)
    x = synth.items(64, 77, dev)
    for _ in range(a.calls):
        rq.get_indices(x)
    torch.cuda.synchronize()
if "pred128" in what:   # predict(seqs[128]) at C3 weights (SASRec/evaluate.py:13, 26)
    sm = synth.sasrec_model(100_000, synth.sasrec_params(64, 50, 2, 1, 64, dev), dev)
    seqs = synth.sequences(128, 50, 100_000, 78, dev)
    for _ in range(a.calls):
        sm.predict(seqs)
    torch.cuda.synchronize()
if "rank128" in what:   # evaluate.rank_batch at batch 128 (SASRec/evaluate.py:26-32 without logits)
    from gr_amd import evaluate as E
    sm = synth.sasrec_model(100_000, synth.sasrec_params(64, 50, 2, 1, 64, dev), dev)
    seqs = synth.sequences(128, 50, 100_000, 78, dev)
    tg = torch.randint(1, 100_001, (128,), generator=torch.Generator(device=dev).manual_seed(9), device=dev)
    for _ in range(a.calls):
        E.rank_batch(sm, seqs, tg)
    torch.cuda.synchronize()
if "c3" in what:   # C3 predict: B 2048, d 64, n 50, 100k items (fused forward + contiguous scoring)
    sm = synth.sasrec_model(100_000, synth.sasrec_params(64, 50, 2, 1, 64, dev), dev)
    seqs = synth.sequences(2048, 50, 100_000, 78, dev)
    for _ in range(a.calls):
        sm.predict(seqs)
    torch.cuda.synchronize()
if "refeval" in what:   # SASRec/evaluate.py at main.py's configuration: d 16, n 20, 706 items, batch 128
    from gr_amd import evaluate as E
    sm = synth.sasrec_model(706, synth.sasrec_params(16, 20, 2, 1, 64, dev), dev, seed=16)
    seqs = synth.sequences(128, 20, 706, 9000, dev)
    tg = torch.randint(1, 707, (128,), generator=torch.Generator(device=dev).manual_seed(9), device=dev)
    for _ in range(a.calls):
        E.rank_batch(sm, seqs, tg)
    torch.cuda.synchronize()
print("done", what, flush=True)
