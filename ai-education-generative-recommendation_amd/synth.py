"""Synthetic workloads of BASELINE.json's configs (no datasets or checkpoints travel to the box).

Item embeddings: ``x = mu + sigma * eps`` with mu/sigma the per-dimension statistics of the 80 real
BERT vectors of stu-major/interaction_records.csv (stored in ``data/bert_stats.npz``), eps ~ N(0,1)
from a seeded device generator.  RQ codebooks are data-derived (k-means-like: residual rows of a
sample plus 1 % noise), as SURVEY §8d prescribes, so the argmin is not dominated by the mass
near-ties of the reference's uniform(+-1/K) init.  SASRec sequences follow the test-mode layout of
SASRec/data_vision.py:74-87 (last n items of the history, left-padded with 0).
"""
import os

import numpy as np
import torch

from . import ops

_STATS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "bert_stats.npz")


def bert_stats():
    z = np.load(_STATS, allow_pickle=False)
    return torch.from_numpy(z["mu"]), torch.from_numpy(z["sigma"])


def items(n, seed, device):
    mu, sigma = bert_stats()
    g = torch.Generator(device=device).manual_seed(seed)
    eps = torch.randn((n, mu.shape[0]), generator=g, device=device, dtype=torch.float32)
    return mu.to(device) + sigma.to(device) * eps


@torch.no_grad()
def rqvae_model(L, K, device, e_dim=32, layers=(256, 128), seed=0, sample=16384):
    """RQVAE with random-init encoder (xavier, seeded) and data-derived codebooks."""
    from .rqvae import RQVAE
    torch.manual_seed(seed)
    m = RQVAE(in_dim=768, num_emb_list=[K] * L, e_dim=e_dim, layers=list(layers), dropout_prob=0.1,
              sk_epsilons=[0.0] * L).to(device).eval()
    g = torch.Generator(device=device).manual_seed(seed + 1)
    for lin in m.encoder.linears():
        lin.bias.copy_(0.01 * torch.randn(lin.bias.shape, generator=g, device=device))
    r = m.encoder(items(sample, seed + 2, device))
    for q in m.rq.vq_layers:
        pick = torch.randint(0, r.shape[0], (K,), generator=g, device=device)
        cb = r[pick] + 0.01 * r.std() * torch.randn((K, r.shape[1]), generator=g, device=device)
        q.embedding.weight.copy_(cb)
        idx = ops.rq_quantize(r, [q.embedding.weight])[:, 0]
        c = q.embedding.weight[idx]
        r = r - (r + (c - r))
    return m


def sasrec_params(d, n, blocks=2, heads=1, mlp=64, device="cuda:0"):
    return {"device": str(device), "d": d, "max_len": n, "num_blocks": blocks, "num_heads": heads,
            "dropout": 0.2, "mlp_layer": mlp, "layernorm_eps": 1e-8}


@torch.no_grad()
def sasrec_model(item_num, params, device, seed=0):
    from .sasrec import SASRec
    torch.manual_seed(seed)
    m = SASRec(item_num, params).to(device).eval()
    g = torch.Generator(device=device).manual_seed(seed + 1)
    for k, v in m.state_dict().items():   # non-trivial biases / LayerNorm affine
        if k.endswith("bias") or "layernorm" in k:
            v.add_(0.05 * torch.randn(v.shape, generator=g, device=device))
    return m


def sequences(B, n, item_num, seed, device):
    """Lengths U[2, n] (U[1, 1] at n = 1), ids U[1, item_num], left-padded with 0."""
    g = torch.Generator(device=device).manual_seed(seed)
    ids = torch.randint(1, item_num + 1, (B, n), generator=g, device=device)
    lens = torch.randint(min(2, n), n + 1, (B, 1), generator=g, device=device)
    pos = torch.arange(n, device=device)[None, :]
    return torch.where(pos >= n - lens, ids, torch.zeros_like(ids))
