"""CPU restatement of RQ-VAE ``get_indices`` (test infrastructure only, see oracle/__init__.py).

Every function follows the reference ATen sequence so that, on the same host, the
outputs are bit-identical to the reference (pinned by tests/test_oracle_golden.py).
"""
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
