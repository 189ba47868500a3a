"""The fused MLP training kernels (csrc/rq_mlp_train.hip, ops.mlp_train) against torch autograd.

MLPLayers in train mode (RQ-VAE/models/layers.py:18-43) is [Dropout -> Linear -> ReLU] x (L - 1),
then Dropout -> Linear.  With dropout 0 the fused forward and backward must match the torch modules'
(fp32 sums in other orders: outputs within 1e-5 and gradients within 2e-5 of their tensor's largest
magnitude).  With dropout on, the kernels draw their own masks (a counter-based hash of the device
seed word, not torch's stream); a one-layer MLP with an identity weight exposes the mask, and the
fused gradients must equal torch autograd's on that same mask.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _mlp(dims, dropout, dev, seed=0):
    from gr_amd.rqvae import MLPLayers
    torch.manual_seed(seed)
    m = MLPLayers(dims, dropout=dropout).to(dev).train()
    for lin in m.linears():   # non-zero biases exercise the bias gradient
        lin.bias.data.normal_(0.0, 0.1)
    return m


def _rel(a, b):
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dims,M", [([768, 256, 128, 32], 64), ([32, 128, 256, 768], 64),
                                    ([768, 256, 128, 32], 200), ([48, 40, 8], 33)])
def test_fused_mlp_matches_torch_without_dropout(dims, M, dev):
    import copy
    m = _mlp(dims, 0.0, dev)
    ref = copy.deepcopy(m)
    ref.fused_train = False
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, dims[0], generator=g, device=dev)
    up = torch.randn(M, dims[-1], generator=g, device=dev)
    outs = []
    for mm in (m, ref):
        xx = x.clone().requires_grad_(True)
        y = mm.train_forward(xx)
        (y * up).sum().backward()
        outs.append((y.detach(), xx.grad))
    assert _rel(outs[0][0], outs[1][0]) <= 1e-5
    assert _rel(outs[0][1], outs[1][1]) <= 2e-5
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) <= 2e-5, k


def test_fused_mlp_dropout_gradients_on_the_kernel_mask(dev):
    from gr_amd import ops
    K, M, p = 96, 70, 0.3
    m = _mlp([K, K], p, dev)
    lin = m.linears()[0]
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.rand(M, K, generator=g, device=dev) + 0.5          # positive: the mask is y / x
    seed = ops.dropout_seed(dev)
    s0 = int(seed.item())
    # the mask of this seed word: identity weight, zero bias
    with torch.no_grad():
        w0, b0 = lin.weight.clone(), lin.bias.clone()
        lin.weight.copy_(torch.eye(K, device=dev))
        lin.bias.zero_()
        seed.fill_(s0)
        keep = ops.mlp_train(x, m) / x
        lin.weight.copy_(w0)
        lin.bias.copy_(b0)
    kept = (keep > 0).float().mean().item()
    assert abs(kept - (1 - p)) < 0.03                               # Bernoulli(1 - p) keeps
    assert torch.allclose(keep[keep > 0], torch.full_like(keep[keep > 0], 1 / (1 - p)))
    up = torch.randn(M, K, generator=g, device=dev)
    seed.fill_(s0)                                                   # the same masks again
    xx = x.clone().requires_grad_(True)
    y = ops.mlp_train(xx, m)
    (y * up).sum().backward()
    x2 = x.clone().requires_grad_(True)
    w2 = lin.weight.detach().clone().requires_grad_(True)
    b2 = lin.bias.detach().clone().requires_grad_(True)
    y2 = F.linear(x2 * keep, w2, b2)
    (y2 * up).sum().backward()
    assert _rel(y.detach(), y2.detach()) <= 1e-5
    assert _rel(xx.grad, x2.grad) <= 2e-5
    assert _rel(lin.weight.grad, w2.grad) <= 2e-5
    assert _rel(lin.bias.grad, b2.grad) <= 2e-5


def test_rqvae_forward_uses_fused_mlps_and_trains(dev):
    """RQVAE.forward in train mode runs the encoder / decoder on the fused kernels (the same
    gradients as the torch modules at dropout 0) and main.py's dropout 0.1 trains."""
    import copy
    from gr_amd import RQVAE
    torch.manual_seed(0)
    m = RQVAE(in_dim=768, num_emb_list=[8, 8, 8], e_dim=32, layers=[256, 128], dropout_prob=0.0,
              quant_loss_weight=0.1, beta=0.25, sk_epsilons=[0.01] * 3, sk_iters=50).to(dev).train()
    for q in m.rq.vq_layers:
        q.embedding.weight.data.normal_(0.0, 0.3)
    ref = copy.deepcopy(m)
    ref.encoder.fused_train = ref.decoder.fused_train = False
    x = torch.randn(64, 768, generator=torch.Generator(device=dev).manual_seed(3), device=dev)
    res = []
    for mm in (m, ref):
        mm.zero_grad(set_to_none=True)
        o, rq_loss, idx = mm(x)
        loss, _ = mm.compute_loss(o, rq_loss, xs=x)
        loss.backward()
        res.append((loss.item(), idx))
    assert torch.equal(res[0][1], res[1][1])
    assert abs(res[0][0] - res[1][0]) <= 1e-5 * abs(res[1][0])
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        assert _rel(p.grad, q.grad) <= 5e-5, k
