"""Fused SASRec training kernels (csrc/sasrec_train.hip, ops._SasTrain) against torch autograd.

The reference's train-mode forward (SASRec/model.py:49-96 as called by SASRec/train.py:131) and its
backward (train.py:161-172) are restated functionally in torch fp32 with the kernels' dropout masks
(reproduced here from the same counter-based hash), so the forward output and the gradient of every
parameter can be compared on the same masks: dropout 0 (plain module semantics) and 0.2 (main.py).
fp32 sums run in different orders on the two sides: outputs within 2e-5 and gradients within 2e-4
of their tensor's max magnitude.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _mix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & M64
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return z ^ (z >> np.uint64(31))


def keep_mask(seed, B, site, count, p):
    """The kernels' keep factors (sasrec_train.hip keep()): [B, count] of 0 or 1 / (1 - p)."""
    if p <= 0:
        return np.ones((B, count), np.float32)
    with np.errstate(over="ignore"):
        idx = np.arange(count, dtype=np.uint64)
        key = (np.uint64(site) << np.uint64(32)) | idx
        inner = _mix64(key)[None, :]
        b = np.arange(B, dtype=np.uint64)[:, None]
        z = _mix64(np.uint64(seed) ^ _mix64(b ^ inner))
    u = (z >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    return np.where(u >= np.float32(p), np.float32(1.0) / np.float32(1.0 - np.float32(p)), 0).astype(np.float32)


def ref_forward(model, seqs, seed, p):
    """model.py:58-96 in torch ops with explicit dropout masks (the kernels' masks)."""
    B, n = seqs.shape
    d, H, m = model.d, model.num_heads, model.mlp_layer
    hd = d // H
    dev = seqs.device
    mk = lambda site, cnt: torch.from_numpy(keep_mask(seed, B, site, cnt, p)).to(dev)   # noqa: E731
    x = F.embedding(seqs, model.item_emb.weight, padding_idx=0) + model.pos_emb.weight[:n][None]
    causal = torch.ones((n, n), dtype=torch.bool, device=dev).triu(1)
    for k, (la, at, lf, ff) in enumerate(zip(model.attention_layernorms, model.attention_layers,
                                             model.forward_layernorms, model.forward_layers)):
        h = F.layer_norm(x, (d,), la.weight, la.bias, model.layernorm_eps)
        qkv = F.linear(h, at.in_proj_weight, at.in_proj_bias)
        q, kk, v = qkv.split(d, dim=-1)
        q = q.view(B, n, H, hd).transpose(1, 2) * (1.0 / hd) ** 0.5
        kk = kk.view(B, n, H, hd).transpose(1, 2)
        v = v.view(B, n, H, hd).transpose(1, 2)
        s = (q @ kk.transpose(-1, -2)).masked_fill(causal, float("-inf"))
        pr = torch.softmax(s, dim=-1) * mk(3 * k, H * n * n).view(B, H, n, n)
        o = (pr @ v).transpose(1, 2).reshape(B, n, d)
        x = x + F.linear(o, at.out_proj.weight, at.out_proj.bias)
        f = F.layer_norm(x, (d,), lf.weight, lf.bias, model.layernorm_eps)
        u = torch.relu(F.linear(f, ff[0].weight, ff[0].bias)) * mk(3 * k + 1, n * m).view(B, n, m)
        x = x + F.linear(u, ff[3].weight, ff[3].bias) * mk(3 * k + 2, n * d).view(B, n, d)
    return F.layer_norm(x, (d,), model.last_layernorm.weight, model.last_layernorm.bias, model.layernorm_eps)


def _close(a, b, tol, what):
    scale = max(float(b.abs().max()), 1e-6)
    err = float((a - b).abs().max())
    assert err <= tol * scale, f"{what}: max |diff| {err:.3e} vs scale {scale:.3e}"


@pytest.mark.parametrize("B,n,d,H,m,nb,p", [
    (6, 20, 16, 1, 64, 2, 0.0),     # main.py's configuration, dropout off
    (6, 20, 16, 1, 64, 2, 0.2),     # main.py's configuration (dropout 0.2)
    (3, 50, 64, 2, 64, 2, 0.2),     # C3 shapes, two heads
    (2, 64, 64, 4, 128, 3, 0.1),    # the kernels' limits: n 64, d 64, mlp 128
])
def test_train_forward_backward_matches_autograd(B, n, d, H, m, nb, p, dev):
    from gr_amd import ops, synth
    prm = synth.sasrec_params(d, n, nb, H, m, dev)
    prm["dropout"] = p
    items = 500
    model = synth.sasrec_model(items, prm, dev, seed=3).train()
    g = torch.Generator(device=dev).manual_seed(5)
    seqs = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    seqs[0, : n // 2] = 0          # left padding (padding row 0 gets no gradient)
    seqs[-1, 3] = seqs[-1, 5]      # a repeated item (its rows' gradients add)
    params = ops._train_params(model)
    seed = int(ops.dropout_seed(dev).item())
    out = model(seqs)
    assert int(ops.dropout_seed(dev).item()) == seed + 1
    ref = ref_forward(model, seqs, seed, p)
    _close(out.detach(), ref.detach(), 2e-5, "forward")
    upstream = torch.randn(out.shape, generator=g, device=dev)
    got = torch.autograd.grad((out * upstream).sum(), params)
    want = torch.autograd.grad((ref * upstream).sum(), params)
    names = ["item_emb", "pos_emb"] + [f"blk{k}.{x}" for k in range(nb) for x in
                                       ("ln_a.w", "ln_a.b", "in_w", "in_b", "out_w", "out_b", "ln_f.w", "ln_f.b",
                                        "ffn1.w", "ffn1.b", "ffn2.w", "ffn2.b")] + ["last.w", "last.b"]
    for name, a, b in zip(names, got, want):
        assert a.shape == b.shape, name
        _close(a, b, 2e-4, name)
    assert float(got[0][0].abs().max()) == 0.0   # padding row
    torch.cuda.synchronize()
    ops.check_errors(dev)


def test_train_module_path_equivalence(dev):
    """fused_train on vs off (the module-by-module autograd path) at dropout 0."""
    import copy
    from gr_amd import synth
    prm = synth.sasrec_params(32, 30, 2, 1, 64, dev)
    prm["dropout"] = 0.0
    a = synth.sasrec_model(300, prm, dev, seed=4).train()
    b = copy.deepcopy(a)
    b.fused_train = False
    seqs = torch.randint(0, 301, (4, 30), generator=torch.Generator(device=dev).manual_seed(1), device=dev)
    ya, yb = a(seqs), b(seqs)
    _close(ya.detach(), yb.detach(), 2e-5, "forward")
    ya.square().sum().backward()
    yb.square().sum().backward()
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        if pb.grad is None:
            assert pa.grad is None, name     # W_Q / W_K / W_V feed nothing (model.py:63-65)
            continue
        _close(pa.grad, pb.grad, 2e-4, name)


def test_train_dropout_rate_and_fresh_masks(dev):
    """Each call draws new masks (the seed word advances) at the configured rate."""
    from gr_amd import synth
    prm = synth.sasrec_params(16, 20, 1, 1, 64, dev)
    prm["dropout"] = 0.2
    model = synth.sasrec_model(100, prm, dev, seed=2).train()
    seqs = torch.randint(1, 101, (8, 20), generator=torch.Generator(device=dev).manual_seed(3), device=dev)
    y1, y2 = model(seqs), model(seqs)
    assert not torch.equal(y1, y2)
    km = keep_mask(12345, 64, 1, 20 * 64, 0.2)
    assert abs(float((km == 0).mean()) - 0.2) < 0.01
