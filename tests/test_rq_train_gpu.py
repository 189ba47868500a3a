"""The captured RQ-VAE training step (ops.RqTrainGraph) against the same step issued eagerly.

RQ-VAE/train.py:108-119 per batch: ``model(data)`` (Sinkhorn assignment of every level on the
kernels, main.py's sk_epsilons 0.01 / sk_iters 50), ``compute_loss``, ``backward``,
``clip_grad_norm_(params, 1.0)``, AdamW (main.py:36-38 lr 1e-3, weight decay 1e-4) under the linear
warm-up schedule (train.py:81-89).  The eager step's gradients are pinned to the reference's own
(tests/test_rq_forward.py); here the graph must reproduce the eager step: with dropout off, loss,
reconstruction loss and indices exact and every parameter within 1e-6 of its largest magnitude after
several replays on different batches; with main.py's dropout, k-means init on the first batch, the
schedule's lr reaching the captured step, and the loss going down.
"""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(dev, dropout, kmeans_init, K=8, seed=0):
    from gr_amd import RQVAE
    torch.manual_seed(seed)
    m = RQVAE(in_dim=768, num_emb_list=[K] * 3, e_dim=32, layers=[256, 128], dropout_prob=dropout,
              bn=False, loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=kmeans_init,
              kmeans_iters=20, sk_epsilons=[0.01] * 3, sk_iters=50)
    if not kmeans_init:   # data-scale codebooks instead of uniform(+-1/K)
        for q in m.rq.vq_layers:
            q.embedding.weight.data.normal_(0.0, 0.3)
    return m.to(dev).train()


def _opt(m, dev, total=100, warm=5, fused=None):
    # fused=None is torch's default AdamW; an explicit fused=False with capturable=True and a tensor
    # lr turns every parameter into NaN at the schedule's lr-0 step on this torch build, with or
    # without the gr_amd kernels (scripts/diag_rq_nan.py), so the tests use the default and fused
    from transformers import get_linear_schedule_with_warmup
    opt = torch.optim.AdamW(m.parameters(), lr=torch.tensor(1e-3, device=dev), weight_decay=1e-4,
                            capturable=True, fused=fused)
    return opt, get_linear_schedule_with_warmup(opt, warm, total)


def _batches(dev, n, B=64, seed=3):
    g = torch.Generator(device=dev).manual_seed(seed)
    mu = torch.randn(768, generator=g, device=dev) * 0.5
    return [mu + 0.3 * torch.randn(B, 768, generator=g, device=dev) for _ in range(n)]


@pytest.mark.parametrize("fused", [None, True], ids=["default_adamw", "fused_adamw"])
def test_graph_step_equals_eager_step(fused, dev):
    from gr_amd import ops
    m = _model(dev, 0.0, False)
    ref = copy.deepcopy(m)
    opt, sch = _opt(m, dev, warm=1, fused=fused)
    ropt, rsch = _opt(ref, dev, warm=1, fused=fused)
    data = _batches(dev, 4)
    inputs = data[0].clone()
    step = ops.RqTrainGraph(m, opt, inputs)
    for x in data:
        inputs.copy_(x)
        loss, recon, idx = step.replay()
        sch.step()
        ropt.zero_grad(set_to_none=True)
        o, rq_loss, ridx = ref(x)
        rloss, rrecon = ref.compute_loss(o, rq_loss, xs=x)
        rloss.backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        ropt.step()
        rsch.step()
        assert torch.equal(idx, ridx)
        assert loss.item() == rloss.item() and recon.item() == rrecon.item()
    worst = 0.0
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        err = ((p - q).abs().max() / q.abs().max().clamp_min(1e-30)).item()
        worst = max(worst, err)
        assert err <= 1e-6, (k, err)
    print(f"\nRqTrainGraph vs eager after {len(data)} steps: worst scaled parameter difference {worst:.3g}")


def test_graph_step_dropout_kmeans_schedule(dev):
    """main.py's configuration: dropout 0.1, k-means init (done by the constructor on the first
    batch), lr 0 at the first warm-up step (the parameters do not move), then the scheduled lr
    (they do); the reconstruction loss falls over 40 steps on a fixed batch."""
    from gr_amd import ops
    m = _model(dev, 0.1, True)
    opt, sch = _opt(m, dev, total=200, warm=5)
    x = _batches(dev, 1)[0]
    inputs = x.clone()
    step = ops.RqTrainGraph(m, opt, inputs)
    assert all(q.initted and torch.count_nonzero(q.embedding.weight) > 0 for q in m.rq.vq_layers)
    before = [p.detach().clone() for p in m.parameters()]
    loss, recon, idx = step.replay()          # warm-up step 0: lr = 0
    assert all(torch.equal(a, p) for a, p in zip(before, m.parameters()))
    assert idx.shape == (64, 3) and int(idx.min()) >= 0 and int(idx.max()) < 8
    sch.step()
    first = recon.item()
    losses = []
    for _ in range(40):
        loss, recon, idx = step.replay()
        sch.step()
        losses.append(recon.item())
    assert not all(torch.equal(a, p) for a, p in zip(before, m.parameters()))
    assert all(v == v for v in losses)        # finite
    assert losses[-1] < first, (first, losses[-1])


@pytest.mark.parametrize("K,use_sk", [(8, True), (256, True), (256, False)])
def test_fused_quantizer_equals_level_by_level(K, use_sk, dev):
    """ops.rq_quantize_train (one launch forward, two backward) against the level-by-level path
    (kernel assignment, torch values / losses / autograd): indices exact, outputs and losses within
    1e-6, every parameter gradient within 1e-5 of its largest magnitude (torch accumulates the
    straight-through zero terms, (g + a) - a, with rounding; the fused backward does not)."""
    m = _model(dev, 0.0, False, K=K)
    ref = copy.deepcopy(m)
    ref.rq.fused_train = False
    x = _batches(dev, 1, B=200)[0]
    outs = []
    for mm in (m, ref):
        mm.zero_grad(set_to_none=True)
        o, rq_loss, idx = mm(x, use_sk=use_sk)
        loss, _ = mm.compute_loss(o, rq_loss, xs=x)
        loss.backward()
        outs.append((o.detach(), rq_loss.detach(), idx))
    assert torch.equal(outs[0][2], outs[1][2])
    assert (outs[0][0] - outs[1][0]).abs().max() <= 1e-6 * outs[1][0].abs().max()
    assert abs(outs[0][1].item() - outs[1][1].item()) <= 1e-6 * abs(outs[1][1].item())
    for (k, p), (_, q) in zip(m.named_parameters(), ref.named_parameters()):
        err = ((p.grad - q.grad).abs().max() / q.grad.abs().max().clamp_min(1e-30)).item()
        assert err <= 1e-5, (k, err)


def test_graph_replays_back_to_back_equal_synchronised(dev):
    """The kernel path's captured step replays without a host synchronisation: 60 back-to-back
    training replays end in the same parameters, bit for bit, as 60 replays each followed by a
    device synchronisation."""
    from gr_amd import ops
    base = _model(dev, 0.0, False)
    x = _batches(dev, 1)[0]
    res = []
    for sync in (True, False):
        m = copy.deepcopy(base)
        opt, _ = _opt(m, dev, warm=0, total=100000, fused=True)
        step = ops.RqTrainGraph(m, opt, x.clone())
        assert step.graph is not None   # kernel path: captured
        for _ in range(60):
            step.replay()
            if sync:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        res.append([p.detach().clone() for p in m.parameters()])
    assert all(torch.equal(a, b) for a, b in zip(*res))


def test_module_fallback_runs_eagerly_and_matches(dev):
    """fused_train = False (torch modules): the step is not captured (see SasTrainGraph.replay) and
    back-to-back replays equal the same steps issued by hand."""
    from gr_amd import ops
    base = _model(dev, 0.0, False)
    for mod in (base.encoder, base.decoder, base.rq):
        mod.fused_train = False
    data = _batches(dev, 3)
    m, ref = copy.deepcopy(base), copy.deepcopy(base)
    opt, _ = _opt(m, dev, warm=0, total=100000, fused=True)
    ropt, _ = _opt(ref, dev, warm=0, total=100000, fused=True)
    inputs = data[0].clone()
    step = ops.RqTrainGraph(m, opt, inputs)
    assert step.graph is None
    for x in data:
        inputs.copy_(x)
        loss, recon, idx = step.replay()
        ropt.zero_grad(set_to_none=True)
        o, rq_loss, ridx = ref(x)
        rloss, _ = ref.compute_loss(o, rq_loss, xs=x)
        rloss.backward()
        torch.nn.utils.clip_grad_norm_(ref.parameters(), 1.0)
        ropt.step()
        assert torch.equal(idx, ridx) and loss.item() == rloss.item()
    assert all(torch.equal(a, b) for a, b in zip(m.parameters(), ref.parameters()))


def test_capture_restores_module_buffers(dev):
    """bn=True: the warm-up and capture forwards are train-mode BatchNorm steps; the graph's
    constructor must leave running_mean / running_var / num_batches_tracked as it found them
    (ADVICE r2), as it does the parameters and the optimizer state."""
    from gr_amd import RQVAE, ops
    torch.manual_seed(0)
    m = RQVAE(in_dim=768, num_emb_list=[8] * 3, e_dim=32, layers=[256, 128], dropout_prob=0.0, bn=True,
              sk_epsilons=[0.01] * 3, sk_iters=50).to(dev).train()
    for q in m.rq.vq_layers:
        q.embedding.weight.data.normal_(0.0, 0.3)
    before = [b.detach().clone() for b in m.buffers()]
    assert len(before) > 0
    opt, _ = _opt(m, dev)
    ops.RqTrainGraph(m, opt, _batches(dev, 1)[0].clone(), capture=True)
    assert all(torch.equal(a, b) for a, b in zip(before, m.buffers()))
