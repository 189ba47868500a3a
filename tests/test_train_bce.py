"""SASRec training-side scoring (SASRec/train.py:131-167).

``ops.sampled_bce_loss`` returns ``(batch_loss, batch_valid_t)`` without forming the
``[B, n, item_num+1]`` score matrix, and backpropagates into the features and the item table.
Parity: against the reference-generated fixtures (features from the reference model, loss block
from the oracle's verbatim restatement, make_golden_train.py) and against the oracle on seeded
inputs.  Bar: ``valid`` exact; ``batch_loss`` within 1e-5 relative; gradients within 1e-5 of the
tensor's largest magnitude (fp32, different summation order; dM accumulates with atomics).
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import sasrec_oracle

TOL = 1e-5
FIXTURES = ["sas_train_main", "sas_train_d64", "sas_train_d128"]


def _inputs(name):
    _, out, meta = gl.load(name)
    t = {k: torch.from_numpy(out[k]) for k in ("feats", "table", "targets", "negs")}
    return t, out, meta


def _scaled_err(got, ref):
    ref = torch.as_tensor(ref, dtype=torch.float32)
    scale = ref.abs().max().clamp_min(1e-30)
    return ((got.detach().cpu() - ref).abs().max() / scale).item()


@pytest.mark.parametrize("name", FIXTURES)
def test_oracle_matches_golden(name):
    t, out, meta = _inputs(name)
    bl, valid, gf, gw = sasrec_oracle.train_loss_grads(t["feats"], t["table"], t["targets"], t["negs"],
                                                      meta["eps"])
    assert valid.item() == float(out["valid"])
    assert abs(bl.item() - float(out["batch_loss"])) <= 1e-6 * abs(float(out["batch_loss"]))
    assert _scaled_err(gf, out["dfeats"]) <= 1e-6
    assert _scaled_err(gw, out["dtable"]) <= 1e-6


def test_oracle_neg_samples_exclude_history():
    rng = np.random.RandomState(3)
    seqs = np.array([[0, 0, 1, 2, 3], [4, 5, 6, 7, 8]])
    negs = sasrec_oracle.neg_samples(seqs, 12, 4, rng).numpy()
    for s, ng in zip(seqs, negs):
        assert len(set(ng)) == 4 and not set(ng) & set(s[s != 0]) and ng.min() >= 1 and ng.max() <= 12


def _run(t, eps, dev):
    from gr_amd import ops
    f = t["feats"].to(dev).requires_grad_(True)
    w = t["table"].to(dev).requires_grad_(True)
    bl, valid = ops.sampled_bce_loss(f, w, t["targets"].to(dev), t["negs"].to(dev), eps)
    v = valid.item()
    loss = bl / v if v > 0 else bl * 0.0
    loss.backward()
    return bl, valid, f.grad, w.grad


@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_sampled_bce_matches_reference(name, dev):
    t, out, meta = _inputs(name)
    bl, valid, gf, gw = _run(t, meta["eps"], dev)
    assert valid.item() == float(out["valid"])
    ref = float(out["batch_loss"])
    assert abs(bl.item() - ref) <= TOL * abs(ref), (bl.item(), ref)
    assert _scaled_err(gf, out["dfeats"]) <= TOL
    assert _scaled_err(gw, out["dtable"]) <= TOL


@pytest.mark.gpu
@pytest.mark.parametrize("B,n,d,items,J", [(128, 50, 64, 20000, 10), (64, 200, 128, 5000, 10),
                                           (33, 7, 32, 100, 1), (5, 3, 48, 50, 3)])
def test_sampled_bce_vs_oracle_seeded(B, n, d, items, J, dev):
    """Seeded inputs at the reference's training shapes (C3: batch 128, n 50, d 64), C5's n 200 /
    d 128, ragged small cases and a d that is not a multiple of 32."""
    g = torch.Generator().manual_seed(B * 1000 + d)
    feats = torch.randn(B, n, d, generator=g) * 0.3
    table = torch.randn(items + 1, d, generator=g) * 0.3
    table[0] = 0
    targets = torch.randint(1, items + 1, (B, n), generator=g)
    lens = torch.randint(0, n + 1, (B,), generator=g)
    targets[torch.arange(n)[None, :] < (n - lens)[:, None]] = 0      # left padding
    negs = sasrec_oracle.neg_samples(np.zeros((B, 1), np.int64), items, J, np.random.RandomState(B))
    t = dict(feats=feats, table=table, targets=targets, negs=negs)
    bl, valid, gf, gw = _run(t, 1e-24, dev)
    rbl, rvalid, rgf, rgw = sasrec_oracle.train_loss_grads(feats, table, targets, negs, 1e-24)
    assert valid.item() == rvalid.item()
    assert abs(bl.item() - rbl.item()) <= TOL * abs(rbl.item())
    assert _scaled_err(gf, rgf) <= TOL
    assert _scaled_err(gw, rgw) <= TOL


@pytest.mark.gpu
def test_sampled_bce_all_padding(dev):
    from gr_amd import ops
    f = torch.randn(4, 6, 16, device=dev, requires_grad=True)
    w = torch.randn(40, 16, device=dev, requires_grad=True)
    tg = torch.zeros(4, 6, dtype=torch.long, device=dev)
    ng = torch.randint(1, 40, (4, 3), device=dev)
    bl, valid = ops.sampled_bce_loss(f, w, tg, ng, 1e-24)
    assert bl.item() == 0.0 and valid.item() == 0.0
    bl.backward()
    assert torch.count_nonzero(f.grad) == 0 and torch.count_nonzero(w.grad) == 0


@pytest.mark.gpu
def test_sampled_bce_accumulates_into_existing_grads(dev):
    """Autograd semantics: the op's gradients add to gradients from other uses of the table (the
    embedding lookup in the reference's forward)."""
    from gr_amd import ops
    t, out, meta = _inputs("sas_train_main")
    w = t["table"].to(dev).requires_grad_(True)
    f = t["feats"].to(dev)
    bl, valid = ops.sampled_bce_loss(f, w, t["targets"].to(dev), t["negs"].to(dev), meta["eps"])
    (bl / valid.item() + w.sum()).backward()
    assert _scaled_err(w.grad - 1.0, out["dtable"]) <= TOL


@pytest.mark.gpu
def test_sampled_bce_bad_ids_flagged(dev):
    from gr_amd import ops
    f = torch.randn(2, 3, 16, device=dev)
    w = torch.randn(10, 16, device=dev)
    tg = torch.ones(2, 3, dtype=torch.long, device=dev)
    ng = torch.full((2, 2), 10, dtype=torch.long, device=dev)
    old = ops.CHECK
    ops.CHECK = True
    try:
        with pytest.raises(IndexError):
            ops.sampled_bce_loss(f, w, tg, ng, 1e-24)
    finally:
        ops.CHECK = old


# ------------------------------------------------------------------ negative sampling (train.py:15-30)

@pytest.mark.gpu
@pytest.mark.parametrize("B,n,items,J", [(128, 50, 100000, 10), (64, 20, 30, 10), (7, 200, 300, 64), (3, 5, 12, 4)])
def test_neg_samples_constraints(B, n, items, J, dev):
    """Every row: num_neg distinct items in [1, item_num], none in the row's non-zero history
    (the setdiff1d + replace=False contract of get_neg_samples)."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(B + n)
    seq = torch.randint(1, items + 1, (B, n), generator=g)
    seq[:, : n // 3] = 0                                     # left padding
    if items >= J + n:
        seq[0] = torch.randperm(items, generator=g)[:n] + 1  # a full history of distinct items
    out = ops.neg_samples(seq.to(dev), items, J, seed=7).cpu().numpy()
    assert out.shape == (B, J)
    for s, ng in zip(seq.numpy(), out):
        assert len(set(ng.tolist())) == J
        assert ng.min() >= 1 and ng.max() <= items
        assert not set(ng.tolist()) & set(s[s != 0].tolist())


@pytest.mark.gpu
def test_neg_samples_uniform_and_seeded(dev):
    """Distribution = uniform over the valid set (chi-square over 20000 rows), random order,
    repeatable for a given seed."""
    from gr_amd import ops
    items, J, B = 20, 3, 20000
    seq = torch.zeros((B, 4), dtype=torch.long)
    seq[:, 0], seq[:, 1] = 5, 17                             # history {5, 17}: 18 valid items
    a = ops.neg_samples(seq.to(dev), items, J, seed=123)
    assert torch.equal(a, ops.neg_samples(seq.to(dev), items, J, seed=123))
    assert not torch.equal(a, ops.neg_samples(seq.to(dev), items, J, seed=124))
    cnt = np.bincount(a.cpu().numpy().ravel(), minlength=items + 1)
    assert cnt[0] == 0 and cnt[5] == 0 and cnt[17] == 0
    valid = [i for i in range(1, items + 1) if i not in (5, 17)]
    exp = B * J / len(valid)
    chi2 = sum((cnt[i] - exp) ** 2 / exp for i in valid)
    assert chi2 < 45.0          # 17 dof: p ~ 3e-4
    first = np.bincount(a[:, 0].cpu().numpy(), minlength=items + 1)[valid]   # each position uniform too
    assert (first.max() - first.min()) < 0.25 * first.mean()


@pytest.mark.gpu
def test_neg_samples_population_too_small(dev):
    from gr_amd import ops
    seq = torch.tensor([[1, 2, 3, 4], [0, 0, 0, 1]], device=dev)
    old = ops.CHECK
    ops.CHECK = True
    try:
        with pytest.raises(ValueError):
            ops.neg_samples(seq, 6, 3)                       # row 0 has 2 valid items
    finally:
        ops.CHECK = old
    with pytest.raises(RuntimeError):
        ops.neg_samples(seq, 2, 3)                           # num_neg > item_num


@pytest.mark.gpu
def test_neg_samples_population_too_small_default_mode(dev):
    """with GR_AMD_CHECK off (the default) an unfillable row still raises ValueError
    (the call synchronises whenever n + num_neg could exceed half the catalog), and the row holds
    -1 ids, never uninitialised memory."""
    from gr_amd import ops
    assert not ops.CHECK
    seq = torch.tensor([[1, 2, 3, 4], [0, 0, 0, 1]], device=dev)
    with pytest.raises(ValueError):
        ops.neg_samples(seq, 6, 3)
    ops.check_errors(dev)                                    # cleared by the raise
    out = ops.neg_samples(seq[1:], 6, 3)                     # row 1 alone: 5 valid items
    assert ((out >= 2) & (out <= 6)).all() and len(set(out[0].tolist())) == 3
    big = torch.randint(1, 100_000, (64, 50), device=dev)    # the common case: no sync, no error
    out = ops.neg_samples(big, 100_000, 10)
    ops.check_errors(dev)
    assert (out >= 1).all()


# ------------------------------------------------------------------ the whole train.py:131-167 step

@pytest.mark.gpu
@pytest.mark.parametrize("name", FIXTURES)
def test_full_training_step_matches_reference(name, dev):
    """Drop-in SASRec in train mode (forward under autograd, dropout 0 for determinism) +
    ops.sampled_bce_loss + backward: every parameter gradient equals the reference model's
    (make_golden_train.py) within 1e-5 of its tensor's largest magnitude."""
    from gr_amd import SASRec, ops
    sd, out, meta = gl.load(name)
    p = dict(meta["params"], device=str(dev))
    m = SASRec(meta["item_num"], p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev).train()
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    f = m(seqs)
    assert f.requires_grad
    assert _scaled_err(f, out["feats"]) <= TOL
    bl, valid = ops.sampled_bce_loss(f, m.item_emb.weight, torch.from_numpy(out["targets"]).to(dev),
                                     torch.from_numpy(out["negs"]).to(dev), meta["eps"])
    (bl / valid.item()).backward()
    worst = 0.0
    for k, prm in m.named_parameters():
        key = f"pgrad/{k}"
        if key not in out:
            assert prm.grad is None or torch.count_nonzero(prm.grad) == 0, k
            continue
        err = _scaled_err(prm.grad, out[key])
        worst = max(worst, err)
        assert err <= TOL, (k, err)
    print(f"\n{name}: worst scaled parameter-grad error {worst:.3g}")
    # eval mode afterwards runs the kernels again, on the same weights
    m.eval()
    with torch.no_grad():
        assert _scaled_err(m(seqs), out["feats"]) <= TOL


@pytest.mark.gpu
def test_neg_samples_device_seed(dev):
    """The device-seeded sampler: keyed by seed ^ *seed_tensor, seed_tensor advanced by one per call;
    equal keys give equal draws, and the draws keep the contract (distinct, in range, off history)."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(11)
    seqs = torch.randint(0, 5000, (64, 50), generator=g).to(dev)
    st = torch.tensor([123], dtype=torch.int64, device=dev)
    a = ops.neg_samples(seqs, 5000, 10, seed_tensor=st)
    assert int(st.item()) == 124
    b = ops.neg_samples(seqs, 5000, 10, seed_tensor=torch.tensor([123], dtype=torch.int64, device=dev))
    c = ops.neg_samples(seqs, 5000, 10, seed_tensor=st)
    assert torch.equal(a, b) and not torch.equal(a, c)
    for x in (a, c):
        assert int(x.min()) >= 1 and int(x.max()) <= 5000
        for row, hist in zip(x.cpu().tolist(), seqs.cpu().tolist()):
            assert len(set(row)) == 10 and not (set(row) & set(hist))


@pytest.mark.gpu
def test_train_step_graph_matches_eager(dev):
    """ops.SasTrainStepGraph replays the step (fresh device-seeded negatives each replay) with the
    results of the same step issued eagerly on the same negatives: loss and valid exact, gradients
    within 1e-6 of their largest magnitude (dM accumulates with atomics)."""
    from gr_amd import ops
    B, n, d, items, J = 32, 20, 64, 3000, 5
    g = torch.Generator(device=dev).manual_seed(7)
    feats = (0.3 * torch.randn(B, n, d, generator=g, device=dev)).requires_grad_(True)
    table = (0.3 * torch.randn(items + 1, d, generator=g, device=dev)).requires_grad_(True)
    targets = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    targets[:, :5] = 0
    inputs = torch.roll(targets, 1, dims=1)
    inputs[:, 0] = 0
    step = ops.SasTrainStepGraph(feats, table, inputs, targets, items, J, 1e-24, seed=99)
    seen = []
    for _ in range(3):
        key = int(step.seed.item())
        bl, valid = step.replay()
        bl, valid = float(bl.detach()), float(valid)
        gf, gt = feats.grad.clone(), table.grad.clone()
        negs = ops.neg_samples(inputs, items, J, seed_tensor=torch.tensor([key], dtype=torch.int64, device=dev))
        seen.append(negs)
        f2 = feats.detach().clone().requires_grad_(True)
        t2 = table.detach().clone().requires_grad_(True)
        bl2, valid2 = ops.sampled_bce_loss(f2, t2, targets, negs, 1e-24)
        (bl2 / valid2).backward()
        assert bl == float(bl2.detach()) and valid == float(valid2)
        assert (gf - f2.grad).abs().max() <= 1e-6 * f2.grad.abs().max()
        assert (gt - t2.grad).abs().max() <= 1e-6 * t2.grad.abs().max()
    assert not torch.equal(seen[0], seen[1])   # fresh negatives per replay


@pytest.mark.gpu
def test_captured_step_inside_training_loop(dev):
    """INTEGRATION.md's recipe: transformer forward, features copied into the graph's static leaf,
    SasTrainStepGraph.replay(), then the transformer backward from feats.grad -- every parameter
    gradient equals the eager step's (on a copy of the model, same negatives) over two consecutive
    steps, so the graph's static .grad buffers are reused."""
    import copy
    from gr_amd import ops, synth
    B, n, d, items, J = 16, 20, 64, 2000, 5
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    p["dropout"] = 0.0
    m = synth.sasrec_model(items, p, dev, seed=3).train()
    ref_m = copy.deepcopy(m)
    g = torch.Generator(device=dev).manual_seed(5)
    seqs = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    seqs[:, :4] = 0
    targets = torch.roll(seqs, -1, dims=1)
    targets[:, -1] = torch.randint(1, items + 1, (B,), generator=g, device=dev)
    targets[seqs == 0] = 0
    feats = torch.zeros(B, n, d, device=dev, requires_grad=True)
    step = ops.SasTrainStepGraph(feats, m.item_emb.weight, seqs, targets, items, J, 1e-24, seed=11)
    for _ in range(2):
        key = int(step.seed.item())
        for q in m.parameters():            # optimizer.zero_grad(set_to_none=False)
            if q.grad is not None:
                q.grad.zero_()
        h = m.forward(seqs)
        with torch.no_grad():
            feats.copy_(h)
        step.replay()
        h.backward(feats.grad)
        negs = ops.neg_samples(seqs, items, J, seed_tensor=torch.tensor([key], dtype=torch.int64, device=dev))
        ref_m.zero_grad(set_to_none=True)
        bl, valid = ops.sampled_bce_loss(ref_m.forward(seqs), ref_m.item_emb.weight, targets, negs, 1e-24)
        (bl / valid).backward()
        for (name, q), r in zip(m.named_parameters(), ref_m.parameters()):
            if r.grad is None:
                assert q.grad is None or float(q.grad.abs().max()) == 0.0, name
                continue
            assert (q.grad - r.grad).abs().max() <= 1e-5 * max(float(r.grad.abs().max()), 1e-30), name


@pytest.mark.gpu
@pytest.mark.parametrize("opt_name", ["sgd", "adam"])
def test_whole_train_step_graph_matches_eager(opt_name, dev):
    """ops.SasTrainGraph (forward + negatives + fused loss + backward + optimizer step, one graph)
    against the same steps issued eagerly on a copy of the model (dropout 0, the same negatives).
    SGD: every parameter after three steps within 1e-5 of its scale (the dM atomics reorder last
    bits).  Adam (the reference's optimizer, train.py:107): per-step losses within 1e-5 relative --
    Adam turns the rounding noise of a mathematically zero gradient (the attention's key bias) into
    +-lr steps, so parameters are compared only through the loss they produce.  Both: the warm-up
    leaves no trace (first replay = step 1) and each replay draws fresh negatives."""
    import copy
    from gr_amd import ops, synth
    B, n, d, items, J = 32, 20, 64, 3000, 5
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    p["dropout"] = 0.0
    m = synth.sasrec_model(items, p, dev, seed=7).train()
    ref = copy.deepcopy(m)
    if opt_name == "sgd":
        opt = torch.optim.SGD(m.parameters(), lr=0.05)
        ref_opt = torch.optim.SGD(ref.parameters(), lr=0.05)
    else:
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, betas=(0.9, 0.98), capturable=True)
        ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-3, betas=(0.9, 0.98))
    g = torch.Generator(device=dev).manual_seed(9)
    seqs = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
    seqs[:, :3] = 0
    targets = torch.roll(seqs, -1, dims=1)
    targets[:, -1] = torch.randint(1, items + 1, (B,), generator=g, device=dev)
    targets[seqs == 0] = 0
    step = ops.SasTrainGraph(m, opt, seqs, targets, items, J, 1e-24, seed=21)
    for a, b in zip(m.parameters(), ref.parameters()):
        assert torch.equal(a, b)   # the warm-up steps were undone
    keys = []
    for _ in range(3):
        key = int(step.seed.item())
        keys.append(key)
        bl, valid = step.replay()
        negs = ops.neg_samples(seqs, items, J, seed_tensor=torch.tensor([key], dtype=torch.int64, device=dev))
        ref_opt.zero_grad()
        bl2, valid2 = ops.sampled_bce_loss(ref(seqs), ref.item_emb.weight, targets, negs, 1e-24)
        (bl2 / valid2).backward()
        ref_opt.step()
        assert float(valid) == float(valid2)
        assert abs(float(bl) - float(bl2.detach())) <= 1e-5 * abs(float(bl2.detach()))
    assert len(set(keys)) == 3
    if opt_name == "sgd":
        with torch.no_grad():
            for (name, a), b in zip(m.named_parameters(), ref.parameters()):
                assert (a - b).abs().max() <= 1e-5 * max(float(b.abs().max()), 1e-6), name
