"""Drop-in SASRec module whose eval forward / full-catalog scoring run on the gfx950 kernels.

Same constructor ``SASRec(item_num, params)``, submodule tree and ``state_dict`` keys as the
reference (SASRec/model.py:6-47), so ``SASRec/evaluate.py`` runs unchanged after swapping

    from model import SASRec                  ->   from gr_amd.sasrec import SASRec

``predict(log_seqs)`` (model.py:98-108) is one C-ABI call (``gr_sasrec_predict_f32``) and returns a
fresh writable ``[B, item_num+1]`` tensor (evaluate.py:27 writes column 0 in place).
"""
import torch
import torch.nn as nn

from . import ops


class SASRec(nn.Module):
    def __init__(self, item_num, params):
        super().__init__()
        self.item_num = item_num
        self.dev = params["device"]
        self.d = params["d"]
        self.mlp_layer = params["mlp_layer"]
        self.dropout = params["dropout"]
        self.layernorm_eps = params["layernorm_eps"]
        self.num_blocks = params["num_blocks"]
        self.num_heads = params["num_heads"]
        self.item_emb = nn.Embedding(item_num + 1, self.d, padding_idx=0)
        self.pos_emb = nn.Embedding(params["max_len"], self.d)
        # model.py:23-25: these projections are computed by the reference but never used; they are
        # kept only so that checkpoints load with identical keys.
        self.W_Q = nn.Linear(self.d, self.d)
        self.W_K = nn.Linear(self.d, self.d)
        self.W_V = nn.Linear(self.d, self.d)
        self.attention_layernorms = nn.ModuleList(
            [nn.LayerNorm(self.d, eps=self.layernorm_eps) for _ in range(self.num_blocks)])
        self.attention_layers = nn.ModuleList(
            [nn.MultiheadAttention(self.d, self.num_heads, self.dropout, batch_first=True)
             for _ in range(self.num_blocks)])
        self.forward_layernorms = nn.ModuleList(
            [nn.LayerNorm(self.d, eps=self.layernorm_eps) for _ in range(self.num_blocks)])
        self.forward_layers = nn.ModuleList([
            nn.Sequential(nn.Linear(self.d, self.mlp_layer), nn.ReLU(), nn.Dropout(self.dropout),
                          nn.Linear(self.mlp_layer, self.d), nn.Dropout(self.dropout))
            for _ in range(self.num_blocks)])
        self.last_layernorm = nn.LayerNorm(self.d, eps=self.layernorm_eps)

    def _binding(self, log_seqs):
        if self.training and self.dropout > 0:
            raise RuntimeError("gr_amd SASRec kernels implement eval mode (dropout off): call .eval()")
        n = log_seqs.shape[-1]
        if n > self.pos_emb.weight.shape[0]:
            raise IndexError(f"sequence length {n} exceeds max_len {self.pos_emb.weight.shape[0]}")
        return ops.sasrec_binding(self)

    def forward(self, log_seqs):
        """model.py:49-96: ``[B, n]`` item ids -> ``[B, n, d]`` final hidden states.

        Eval mode (or grad disabled): one C-ABI call, ``gr_sasrec_forward_f32``, no autograd graph.
        Train mode with grad enabled (the SASRec/train.py:131 call), dropout active: the fused
        training kernels of sasrec_train.hip when the shape fits them (``ops.sasrec_train_forward``:
        one launch forward, one launch backward -- ``gr_sasrec_train_fwd_f32`` /
        ``gr_sasrec_train_bwd_f32``), otherwise the same blocks as torch modules under autograd
        (``fused_train = False`` forces the latter).  The step's scoring, loss and negative sampling
        are kernels too (``ops.sampled_bce_loss``, ``ops.neg_samples``)."""
        if self.training and torch.is_grad_enabled():
            return self._forward_autograd(log_seqs)
        with torch.no_grad():
            return ops.sasrec_forward(self._binding(log_seqs), log_seqs)

    # Train-mode forward on the fused training kernels (ops.sasrec_train_forward: one launch
    # forward, one backward) whenever the shape fits them (n, d <= 64, mlp_layer <= 128); False
    # keeps the module-by-module autograd path below (used by the parity tests as the reference).
    fused_train = True

    def _forward_autograd(self, log_seqs):
        """model.py:58-96 as module calls: E[s] + P[0..n), then per block a pre-LN causal
        self-attention residual and a pre-LN FFN residual, then the last LayerNorm.  The reference's
        W_Q / W_K / W_V outputs (model.py:63-65) feed nothing and are not computed."""
        n = log_seqs.shape[1]
        if n > self.pos_emb.weight.shape[0]:
            raise IndexError(f"sequence length {n} exceeds max_len {self.pos_emb.weight.shape[0]}")
        if self.fused_train and ops.sasrec_train_supported(self, n):
            return ops.sasrec_train_forward(self, log_seqs)
        pos = torch.arange(n, device=log_seqs.device)
        x = self.item_emb(log_seqs) + self.pos_emb(pos).unsqueeze(0)
        causal = torch.ones((n, n), dtype=torch.bool, device=log_seqs.device).triu(1)
        for ln_a, mha, ln_f, ffn in zip(self.attention_layernorms, self.attention_layers,
                                        self.forward_layernorms, self.forward_layers):
            h = ln_a(x)
            x = x + mha(h, h, h, attn_mask=causal)[0]
            x = x + ffn(ln_f(x))
        return self.last_layernorm(x)

    @torch.no_grad()
    def last_hidden(self, log_seqs):
        """``forward(log_seqs)[:, -1, :]`` (model.py:104) without materialising other positions."""
        return ops.sasrec_forward(self._binding(log_seqs), log_seqs, last_only=True)

    # predict's logits layout: True (default) -- a contiguous [B, item_num + 1] tensor like the
    # reference's matmul result (model.py:107; .view() works).  Its rows start anywhere in a 128-byte
    # line; the scoring kernel stores whole lines anyway (lanes rotated by each row's line offset,
    # score.hip score_rot_kernel): 412 vs 393 us per C3 call at B 2048, equal at B <= 512
    # (profiles/r04/ab_predict_contiguous.txt).  False -- a [B, ld] buffer (ld = roundup(item_num +
    # 1, 32)) viewed as [B, item_num + 1]: unit column stride, not contiguous.
    contiguous_logits = True

    @torch.no_grad()
    def predict(self, log_seqs):
        """model.py:98-108: logits ``[B, item_num+1]`` = last hidden state x item table^T, a fresh
        writable contiguous tensor (evaluate.py:27 writes column 0 in place)."""
        out = None
        if self.contiguous_logits:
            out = torch.empty((log_seqs.shape[0], self.item_emb.weight.shape[0]), dtype=torch.float32,
                              device=self.item_emb.weight.device)
        return ops.sasrec_predict(self._binding(log_seqs), log_seqs, out=out)
