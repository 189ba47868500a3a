"""CPU restatement of SASRec forward / predict (test infrastructure only, see oracle/__init__.py).

Follows SASRec/model.py:49-108 and the ``nn.MultiheadAttention`` slow path it takes for an odd
head count (torch/nn/modules/activation.py fast-path gate "num_heads is not even";
torch/nn/functional.py multi_head_attention_forward: packed in-projection :5785-5830, q scaling
:6578, baddbmm with the -inf float mask :6585, softmax :6590, bmm :6594, out-projection :6600).
For even head counts the reference takes ``torch._native_multi_head_attention`` instead; this
restatement then agrees within rounding only (compare with a tolerance).
"""
import math

import numpy as np

import torch
import torch.nn.functional as F


def _mha_slow(x, in_w, in_b, out_w, out_b, num_heads, attn_mask_bool):
    """nn.MultiheadAttention(batch_first=True)(x, x, x, attn_mask=mask)[0] on the slow path."""
    # activation.py: batch_first -> (L, N, E)
    q = x.transpose(1, 0)
    tgt_len, bsz, embed_dim = q.shape
    head_dim = embed_dim // num_heads
    # functional.py _in_projection_packed (self-attention branch)
    proj = F.linear(q, in_w, in_b)
    proj = proj.unflatten(-1, (3, embed_dim)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
    qq, kk, vv = proj[0], proj[1], proj[2]
    # _canonical_mask: bool -> float with -inf where True
    mask = torch.zeros_like(attn_mask_bool, dtype=q.dtype).masked_fill_(attn_mask_bool, float("-inf"))
    mask = mask.unsqueeze(0)
    qq = qq.view(tgt_len, bsz * num_heads, head_dim).transpose(0, 1)
    kk = kk.view(kk.shape[0], bsz * num_heads, head_dim).transpose(0, 1)
    vv = vv.view(vv.shape[0], bsz * num_heads, head_dim).transpose(0, 1)
    q_scaled = qq * math.sqrt(1.0 / float(head_dim))
    w = torch.baddbmm(mask, q_scaled, kk.transpose(-2, -1))
    w = torch.softmax(w, dim=-1)
    o = torch.bmm(w, vv)
    o = o.transpose(0, 1).contiguous().view(tgt_len * bsz, embed_dim)
    o = F.linear(o, out_w, out_b)
    o = o.view(tgt_len, bsz, o.size(1))
    return o.transpose(1, 0)


@torch.no_grad()
def forward(log_seqs, sd, num_blocks, num_heads, eps):
    """SASRec.forward(log_seqs) (SASRec/model.py:49-96) from a reference ``state_dict``.

    ``seqs = M[s] + P[0..n)`` (no sqrt(d) scaling, :58-60); the dead W_Q/W_K/W_V projections
    (:63-65) do not influence the output and are skipped; causal bool mask ``triu(1)`` (:68-69);
    per block pre-LN attention and pre-LN FFN with residuals (:72-94); final LayerNorm (:96).
    """
    seqs = F.embedding(log_seqs, sd['item_emb.weight'], padding_idx=0)
    n = log_seqs.shape[1]
    positions = torch.arange(n).unsqueeze(0).expand_as(log_seqs)
    seqs += F.embedding(positions, sd['pos_emb.weight'])
    d = seqs.shape[-1]
    mask = torch.triu(torch.ones((n, n), dtype=torch.bool), diagonal=1)
    for i in range(num_blocks):
        p = f'attention_layernorms.{i}.'
        h = F.layer_norm(seqs, (d,), sd[p + 'weight'], sd[p + 'bias'], eps)
        a = f'attention_layers.{i}.'
        mha = _mha_slow(h, sd[a + 'in_proj_weight'], sd[a + 'in_proj_bias'],
                        sd[a + 'out_proj.weight'], sd[a + 'out_proj.bias'], num_heads, mask)
        seqs = seqs + mha
        p = f'forward_layernorms.{i}.'
        h = F.layer_norm(seqs, (d,), sd[p + 'weight'], sd[p + 'bias'], eps)
        f = f'forward_layers.{i}.'
        h = F.linear(h, sd[f + '0.weight'], sd[f + '0.bias'])
        h = torch.relu(h)
        h = F.linear(h, sd[f + '3.weight'], sd[f + '3.bias'])
        seqs = seqs + h
    return F.layer_norm(seqs, (d,), sd['last_layernorm.weight'], sd['last_layernorm.bias'], eps)


@torch.no_grad()
def predict(log_seqs, sd, num_blocks, num_heads, eps):
    """SASRec.predict (SASRec/model.py:98-108): ``LN_last(x)[:, -1, :] @ item_emb.weight.t()``."""
    feats = forward(log_seqs, sd, num_blocks, num_heads, eps)
    return feats[:, -1, :].matmul(sd['item_emb.weight'].t())


def neg_samples(seq, item_num, num_neg, rng=np.random):
    """train.py:15-30 get_neg_samples: per row, ``num_neg`` distinct items drawn uniformly from
    ``[1, item_num]`` minus the row's non-zero history (``np.random.choice(..., replace=False)``)."""
    out = []
    for s in np.asarray(seq):
        valid = np.setdiff1d(np.arange(1, item_num + 1), s[s != 0])
        out.append(rng.choice(valid, num_neg, replace=False))
    return torch.tensor(np.array(out), dtype=torch.long)


def train_loss(seq_features, item_emb_weight, target_o_t, negs, eps):
    """train.py:134-158 verbatim in torch (CPU fp32): the full score matrix ``[B, n, N+1]``, the
    target / negative gathers, the masked BCE terms.  Returns ``(batch_loss, batch_valid_t)``;
    autograd through it gives the reference's gradients."""
    score_matrix = torch.matmul(seq_features, item_emb_weight.t())
    mask = (target_o_t != 0).float()
    seq_len = score_matrix.shape[1]
    neg_expanded = negs.unsqueeze(1).expand(-1, seq_len, -1)
    pos_scores = torch.gather(score_matrix, dim=2, index=target_o_t.unsqueeze(-1)).squeeze(-1)
    neg_scores = torch.gather(score_matrix, dim=2, index=neg_expanded)
    pos_loss = -torch.log(torch.sigmoid(pos_scores) + eps) * mask
    neg_loss = (-torch.log(1 - torch.sigmoid(neg_scores) + eps) * mask.unsqueeze(-1)).sum(dim=-1)
    return (pos_loss + neg_loss).sum(), mask.sum()


def train_loss_grads(seq_features, item_emb_weight, target_o_t, negs, eps):
    """``loss = batch_loss / batch_valid_t; loss.backward()`` (train.py:161-167) on the restatement:
    returns ``(batch_loss, valid, d seq_features, d item_emb_weight)``."""
    f = seq_features.detach().clone().requires_grad_(True)
    w = item_emb_weight.detach().clone().requires_grad_(True)
    bl, valid = train_loss(f, w, target_o_t, negs, eps)
    loss = bl / valid.item() if valid.item() > 0 else torch.zeros((), requires_grad=True)
    loss.backward()
    gf = f.grad if f.grad is not None else torch.zeros_like(f)
    gw = w.grad if w.grad is not None else torch.zeros_like(w)
    return bl.detach(), valid, gf, gw
