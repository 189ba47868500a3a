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


def _mix31(x):
    """A 31-bit integer hash (xorshift-multiply rounds; every product stays below 2^63)."""
    for _ in range(3):
        x = ((x ^ (x >> 15)) * 0x2C1B3C6D) & 0x7FFFFFFF
        x = ((x ^ (x >> 12)) * 0x297A2D39) & 0x7FFFFFFF
    return x ^ (x >> 15)


@torch.no_grad()
def table_rows(ids, d, seed, device):
    """Rows ``ids`` of a synthetic item table whose every element is a function of (seed, row, col)
    alone: N(0, 1) by Box-Muller from two 31-bit hashes, row 0 zero (``padding_idx=0``).  Any rank
    can therefore build exactly the rows it needs -- its catalog shard, the rows its users' histories
    gather -- and they agree bit for bit with every other rank's and with any world size's."""
    ids = ids.to(device=device, dtype=torch.int64)
    col = torch.arange(d, device=device, dtype=torch.int64)
    key = (ids[:, None] * d + col[None, :]) & 0x7FFFFFFF
    s = (seed * 0x9E3779B1) & 0x7FFFFFFF
    u1 = (_mix31(key ^ s).to(torch.float64) + 0.5) / 2147483648.0
    u2 = (_mix31(_mix31(key) ^ s ^ 0x5BD1E995).to(torch.float64) + 0.5) / 2147483648.0
    z = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(2.0 * np.pi * u2)
    return torch.where(ids[:, None] == 0, 0.0, z).to(torch.float32)


@torch.no_grad()
def sasrec_rank_model(item_num, params, seqs, device, seed=0, table_seed=7):
    """C5 per-rank model: the transformer parameters of ``sasrec_model`` (independent of the catalog
    size) and an item table holding only the rows ``seqs`` gathers, taken from ``table_rows``.
    Returns (model, seqs remapped into its compact table).  The compact model's hidden states equal
    those of the full ``item_num``-row model built from the same ``table_rows``, bit for bit (the
    forward reads the gathered rows, nothing else of the table)."""
    from .sasrec import SASRec
    torch.manual_seed(seed)
    m = SASRec(1, params).to(device).eval()
    g = torch.Generator(device=device).manual_seed(seed + 1)
    for k, v in m.state_dict().items():
        if k.endswith("bias") or "layernorm" in k:
            v.add_(0.05 * torch.randn(v.shape, generator=g, device=device))
    used = torch.unique(torch.cat([torch.zeros(1, dtype=seqs.dtype, device=seqs.device), seqs.reshape(-1)]))
    if int(used[-1]) > item_num:
        raise IndexError("sequence id beyond the catalog")
    m.item_emb = torch.nn.Embedding(used.numel(), m.d, padding_idx=0).to(device)
    m.item_emb.weight.copy_(table_rows(used, m.d, table_seed, device))
    m.item_num = used.numel() - 1
    return m.eval(), torch.searchsorted(used, seqs)


def sequences(B, n, item_num, seed, device):
    """Lengths U[2, n] (U[1, 1] at n = 1), ids U[1, item_num], left-padded with 0."""
    g = torch.Generator(device=device).manual_seed(seed)
    ids = torch.randint(1, item_num + 1, (B, n), generator=g, device=device)
    lens = torch.randint(min(2, n), n + 1, (B, 1), generator=g, device=device)
    pos = torch.arange(n, device=device)[None, :]
    return torch.where(pos >= n - lens, ids, torch.zeros_like(ids))
