"""CPU restatement of RQ-VAE ``get_indices`` (test infrastructure only, see oracle/__init__.py).

Every function follows the reference ATen sequence so that, on the same host, the
outputs are bit-identical to the reference (pinned by tests/test_oracle_golden.py).
"""
import numpy as np
import torch


def mlp_encode(x, weights, biases):
    """MLPLayers.forward in eval mode (RQ-VAE/models/layers.py:18-33, 42-43).

    ``[Dropout -> Linear -> ReLU] * (len-2)`` then ``Dropout -> Linear`` (no activation after the
    last Linear, layers.py:28-30).  Dropout is the identity in eval mode.  ``nn.Linear`` is
    ``addmm(b, x, W^T)`` (torch.nn.functional.linear).
    """
    h = x
    n = len(weights)
    for i, (w, b) in enumerate(zip(weights, biases)):
        h = torch.nn.functional.linear(h, w, b)
        if i != n - 1:
            h = torch.relu(h)
    return h


def vq_level(latent, codebook):
    """VectorQuantizer.forward(x, use_sk=False) (RQ-VAE/models/vq.py:63-99).

    Returns (x_q, indices, d) where ``d`` is the distance matrix exactly as vq.py:71-73 forms it:
    ``(sum(r**2) + sum(C**2).t()) - 2 * (r @ C.t())``; ``argmin`` returns the first minimum (vq.py:75);
    ``x_q = r + (C[idx] - r)`` is the straight-through expression of vq.py:95.
    """
    d = torch.sum(latent ** 2, dim=1, keepdim=True) + \
        torch.sum(codebook ** 2, dim=1, keepdim=True).t() - \
        2 * torch.matmul(latent, codebook.t())
    indices = torch.argmin(d, dim=-1)
    x_q = torch.nn.functional.embedding(indices, codebook)
    x_q = latent + (x_q - latent)
    return x_q, indices, d


def rq_quantize(z, codebooks, return_detail=False):
    """ResidualVectorQuantizer.forward(x, use_sk=False) (RQ-VAE/models/rq.py:39-56).

    ``residual <- residual - x_res`` per level (rq.py:47); indices stacked on the last dim (rq.py:54).
    With ``return_detail`` also returns per-level residual inputs and the per-row gap between the best
    and second-best fp32 distance at every level (used to certify near-ties).
    """
    residual = z
    idx, residuals, gaps = [], [], []
    for cb in codebooks:
        x_res, ind, d = vq_level(residual, cb)
        if return_detail:
            residuals.append(residual.clone())
            top2 = torch.topk(d, k=min(2, d.shape[1]), dim=1, largest=False).values
            gap = (top2[:, 1] - top2[:, 0]) if d.shape[1] > 1 else torch.full_like(top2[:, 0], float("inf"))
            gaps.append(gap)
        residual = residual - x_res
        idx.append(ind)
    out = torch.stack(idx, dim=-1)
    if return_detail:
        return out, residuals, torch.stack(gaps, dim=-1)
    return out


@torch.no_grad()
def get_indices(x, weights, biases, codebooks, batch_size=None):
    """RQVAE.get_indices(xs, use_sk=False) (RQ-VAE/models/rqvae.py:67-71).

    ``batch_size`` reproduces the caller's DataLoader chunking (RQ-VAE/infer.py:84-95 uses 64):
    the CPU bits of the encoder GEMM depend on the batch size for tiny batches.
    """
    if batch_size is None:
        return rq_quantize(mlp_encode(x, weights, biases), codebooks)
    outs = [rq_quantize(mlp_encode(x[i:i + batch_size], weights, biases), codebooks)
            for i in range(0, x.shape[0], batch_size)]
    return torch.cat(outs, 0)


def state_to_lists(state_dict, n_levels):
    """Split an ``RQVAE.state_dict()`` into encoder weights/biases and codebooks.

    Keys follow RQ-VAE/models/layers.py:18-33 (``encoder.mlp_layers.{1,4,7,..}``: Dropout sits at the
    even indices, ReLU after each non-final Linear) and vq.py:22 (``rq.vq_layers.{l}.embedding.weight``).
    """
    lin = sorted({int(k.split('.')[2]) for k in state_dict if k.startswith('encoder.mlp_layers.')
                  and k.endswith('.weight')})
    ws = [state_dict[f'encoder.mlp_layers.{i}.weight'] for i in lin]
    bs = [state_dict[f'encoder.mlp_layers.{i}.bias'] for i in lin]
    cbs = [state_dict[f'rq.vq_layers.{l}.embedding.weight'] for l in range(n_levels)]
    return ws, bs, cbs


# ----------------------------------------------------------------------------- use_sk=True
def center_distance(d):
    """VectorQuantizer.center_distance_for_constraint (RQ-VAE/models/vq.py:52-61)."""
    mx, mn = d.max(), d.min()
    middle = (mx + mn) / 2
    amplitude = mx - middle + 1e-5
    assert amplitude > 0
    return (d - middle) / amplitude


@torch.no_grad()
def sinkhorn(distances, epsilon, iters):
    """sinkhorn_algorithm (RQ-VAE/models/layers.py:85-108), float64 input."""
    Q = torch.exp(- distances / epsilon)
    B, K = Q.shape
    Q /= Q.sum(-1, keepdim=True).sum(-2, keepdim=True)
    for _ in range(iters):
        Q /= torch.sum(Q, dim=1, keepdim=True)
        Q /= B
        Q /= torch.sum(Q, dim=0, keepdim=True)
        Q /= K
    Q *= B
    return Q


def vq_level_sk(latent, codebook, sk_epsilon, sk_iters):
    """VectorQuantizer.forward(x, use_sk=True) (vq.py:63-99): Sinkhorn assignment when
    sk_epsilon > 0 (vq.py:76-84), else the argmin path."""
    if sk_epsilon <= 0:
        x_q, ind, _ = vq_level(latent, codebook)
        return x_q, ind
    d = torch.sum(latent ** 2, dim=1, keepdim=True) + \
        torch.sum(codebook ** 2, dim=1, keepdim=True).t() - \
        2 * torch.matmul(latent, codebook.t())
    d = center_distance(d).double()
    Q = sinkhorn(d, sk_epsilon, sk_iters)
    ind = torch.argmax(Q, dim=-1)
    x_q = torch.nn.functional.embedding(ind, codebook)
    return latent + (x_q - latent), ind


@torch.no_grad()
def get_indices_sk(x, weights, biases, codebooks, sk_epsilons, sk_iters):
    """RQVAE.get_indices(xs, use_sk=True) (rqvae.py:67-71 -> rq.py:39-56 with vq_level_sk)."""
    residual = mlp_encode(x, weights, biases)
    idx = []
    for cb, eps in zip(codebooks, sk_epsilons):
        x_res, ind = vq_level_sk(residual, cb, eps, sk_iters)
        residual = residual - x_res
        idx.append(ind)
    return torch.stack(idx, dim=-1)


def collision_groups(codes):
    """get_collision_item (RQ-VAE/infer.py:29-41): rows sharing a code, groups in order of the
    code's first appearance, members in row order."""
    index2id = {}
    for i, c in enumerate(map(tuple, np.asarray(codes).tolist())):
        index2id.setdefault(c, []).append(i)
    return [g for g in index2id.values() if len(g) > 1]


def dedup_codes(codes):
    """infer.py:139-162: append a zero column, then number the members of every duplicate code."""
    codes_array = np.hstack((np.asarray(codes), np.zeros((len(codes), 1), dtype=int)))
    unique_codes, counts = np.unique(codes_array, axis=0, return_counts=True)
    for duplicate in unique_codes[counts > 1]:
        for i, idx in enumerate(np.where((codes_array == duplicate).all(axis=1))[0]):
            codes_array[idx, -1] = i
    return codes_array


@torch.no_grad()
def infer_codes(x, weights, biases, codebooks, sk_epsilons, sk_iters, batch_size=64, max_rounds=30,
                re_encode=None):
    """infer.py:88-162 without the file writes: codes (batch_size chunks, use_sk=False), collision
    rounds (every level but the last with sk_epsilon 0, infer.py:108-130), dedup digit.
    ``re_encode(rows) -> [g, L]`` overrides the group re-encode (default: get_indices_sk)."""
    codes = get_indices(x, weights, biases, codebooks, batch_size=batch_size).numpy()
    eps = [0.0] * (len(codebooks) - 1) + [sk_epsilons[-1]]
    rounds = []
    for _ in range(max_rounds):
        groups = collision_groups(codes)
        if not groups:
            break
        rounds.append(groups)
        for g in groups:
            out = (re_encode(g) if re_encode is not None else
                   get_indices_sk(x[g], weights, biases, codebooks, eps, sk_iters).numpy())
            codes[g] = out
    return codes, dedup_codes(codes), rounds
