"""SASRec at BASELINE's full catalog sizes against the CPU oracle (the full-size C3 /
C5 parity had been HIP-vs-HIP).

A real ``SASRec`` with the bench's weights (``synth.sasrec_model``) scores the bench's sequences on
the GPU at the bench batch; a sample of users is then recomputed by ``oracle/sasrec_oracle.predict``
(SASRec/model.py:98-108) on the host and compared:

* logits: ``|gpu - oracle| <= 1e-5 * max|row|`` (north_star's tolerance, row-scaled);
* ranks (SASRec/evaluate.py:27-32): exact for every user whose oracle target logit has no
  competitor within 2 delta (delta = 1e-5 row scale, the logits bar); every user's GPU rank lies
  in the band the logits bar allows, ``#{l > t + 2 delta} + 1 <= rank <= #{l > t - 2 delta} + 1``;
* top-10 (C5, ``dist.sharded_rank_topk`` and an 8-shard merge on one GPU): values within delta of
  the oracle's value for the same id, ids equal to the oracle's top-10 wherever consecutive oracle
  values are more than 2 delta apart, and always inside ``{j : l_j >= v_10 - 2 delta}``.
"""
import numpy as np
import pytest
import torch

from oracle import sasrec_oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _oracle(model, seqs_cpu):
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    return sasrec_oracle.predict(seqs_cpu, sd, model.num_blocks, model.num_heads, model.layernorm_eps)


def _targets(ref, seed):
    """Half the users' targets from the oracle's top-20 (non-trivial HR), half uniform."""
    g = np.random.default_rng(seed)
    lg = ref.clone()
    lg[:, 0] = -1e9
    top20 = torch.topk(lg, 20, dim=1).indices.numpy()
    B, rows = ref.shape
    return torch.from_numpy(np.where(g.random(B) < 0.5, top20[np.arange(B), g.integers(0, 20, B)],
                                     g.integers(1, rows, B)).astype(np.int64))


def _rank_bands(ref, targets, delta):
    lg = ref.double().clone()
    lg[:, 0] = -1e9
    t = lg.gather(1, targets[:, None])
    exact = ((lg > t).sum(1) + 1).numpy()
    lo = ((lg > t + 2 * delta[:, None]).sum(1) + 1).numpy()
    hi = ((lg > t - 2 * delta[:, None]).sum(1) + 1).numpy()     # counts the target itself: +1 slack
    isolated = lo == hi - 1                                      # only the target in the band
    return exact, lo, hi, isolated


def _check_logits(got, ref):
    scale = ref.abs().amax(1)
    err = ((got - ref).abs().amax(1) / scale)
    return float(err.max()), scale * TOL


def _check_ranks(ranks, ref, targets, delta):
    exact, lo, hi, iso = _rank_bands(ref, targets, delta)
    assert ((ranks >= lo) & (ranks <= hi)).all(), (ranks, lo, hi)
    assert np.array_equal(ranks[iso], exact[iso])
    return exact, iso


def _check_topk(v, i, ref, delta, k=10):
    lg = ref.double().clone()
    lg[:, 0] = -1e9
    ov, oi = torch.sort(lg, dim=1, descending=True, stable=True)
    ov, oi = ov[:, :k + 1], oi[:, :k + 1]
    v, i = v.double().cpu(), i.cpu()
    n_exact = 0
    for b in range(lg.shape[0]):
        vb = lg[b, i[b]]                                        # oracle value at the GPU's ids
        assert (vb - v[b]).abs().max() <= delta[b], b
        assert (vb >= ov[b, k - 1] - 2 * delta[b]).all(), b      # inside the top-k band
        gaps = ov[b, :k] - ov[b, 1:k + 1]
        if (gaps > 2 * delta[b]).all():
            assert torch.equal(i[b], oi[b, :k]), b
            n_exact += 1
    return n_exact


def test_c3_full_catalog_vs_oracle(dev, parity_log):
    """C3: 2 blocks, d 64, n 50, 100,001-row table; the bench's 2048-user batch on the GPU, 16 users
    (first 8, last 8) through the oracle."""
    from gr_amd import evaluate, ops, synth
    items, n, B = 100_000, 50, 2048
    model = synth.sasrec_model(items, synth.sasrec_params(64, n, 2, 1, 64, dev), dev)
    seqs = synth.sequences(B, n, items, 2000, dev)
    pick = torch.cat([torch.arange(0, 8), torch.arange(B - 8, B)])
    logits = model.predict(seqs)
    got = logits[pick.to(dev)].cpu()
    ref = _oracle(model, seqs[pick.to(dev)].cpu())
    err, delta = _check_logits(got, ref)
    targets = _targets(ref, 3)
    tg_all = torch.randint(1, items + 1, (B,), device=dev)
    tg_all[pick.to(dev)] = targets.to(dev)
    r_mat = ops.rank(logits, tg_all)[pick.to(dev)].cpu().numpy()
    r_fused = evaluate.rank_batch(model, seqs, tg_all)[pick.to(dev)].cpu().numpy()
    exact, iso = _check_ranks(r_mat, ref, targets, delta)
    assert np.array_equal(r_fused, r_mat)
    parity_log(kind="sasrec_full_size", config="C3 (100,001 rows, d 64, n 50)", users=len(pick),
               max_row_scaled_logit_err=err, ranks_exact=int((r_mat == exact).sum()),
               ranks_isolated=int(iso.sum()), hr10_oracle=float((exact <= 10).mean()),
               hr10_gpu=float((r_mat <= 10).mean()))
    assert err <= TOL


def test_c5_full_catalog_vs_oracle(dev, parity_log):
    """C5: d 128, n 200, 1,000,001-row table; the bench's 512 users through the GPU transformer,
    8 users (first 4, last 4) through the oracle; predict logits, the single-shard and the 8-shard
    catalog-sharded rank + top-10."""
    from gr_amd import dist as D, ops, synth
    items, n, B, k = 1_000_000, 200, 512, 10
    model = synth.sasrec_model(items, synth.sasrec_params(128, n, 2, 1, 64, dev), dev, seed=5)
    seqs = synth.sequences(B, n, items, 5000, dev)
    pick = torch.cat([torch.arange(0, 4), torch.arange(B - 4, B)]).to(dev)
    h_all = model.last_hidden(seqs)
    h = h_all[pick]
    got = model.predict(seqs[pick]).cpu()
    ref = _oracle(model, seqs[pick].cpu())
    err, delta = _check_logits(got, ref)
    assert torch.equal(ops.score(h, model.item_emb.weight.detach()), model.predict(seqs[pick]))
    targets = _targets(ref, 7)
    table = model.item_emb.weight.detach()
    rank1, v1, i1 = D.sharded_rank_topk(h, table, 0, targets.to(dev), k=k)
    exact, iso = _check_ranks(rank1.cpu().numpy(), ref, targets, delta)
    n_exact1 = _check_topk(v1, i1, ref, delta, k)
    # 8 catalog shards on one GPU: the per-rank kernels of the 8-GPU run, merged as dist._exchange
    rows = items + 1
    tg = targets.to(dev)
    ts = torch.zeros(len(pick), device=dev)
    shards = [D.shard_range(rows, r, 8) for r in range(8)]
    for lo, hi in shards:
        own = (tg >= lo) & (tg < hi)
        loc = torch.where(own, tg - lo, torch.zeros_like(tg))
        ts += torch.where(own, ops.score_pairs(h, table[lo:hi], loc, mask_col0=(lo == 0)), torch.zeros_like(ts))
    cnt = torch.zeros(len(pick), dtype=torch.int64, device=dev)
    vs, is_ = [], []
    for lo, hi in shards:
        v, i, c = ops.score_topk(h, table[lo:hi], k, lo, thresholds=ts, mask_col0=(lo == 0))
        cnt += c
        vs.append(v)
        is_.append(i)
    v8, i8 = D.merge_topk(torch.cat(vs, 1), torch.cat(is_, 1), k)
    assert torch.equal(cnt + 1, rank1) and torch.equal(v8, v1) and torch.equal(i8, i1)
    parity_log(kind="sasrec_full_size", config="C5 (1,000,001 rows, d 128, n 200)", users=len(pick),
               max_row_scaled_logit_err=err, ranks_exact=int((rank1.cpu().numpy() == exact).sum()),
               ranks_isolated=int(iso.sum()), top10_exact_users=n_exact1,
               hr10_oracle=float((exact <= 10).mean()))
    assert err <= TOL


def test_c5_per_rank_construction_matches_full_table(dev):
    """bench.py's C5 leg builds, per rank, only its catalog shard and the table rows its own users
    gather (synth.sasrec_rank_model).  The hidden states of every world size's user shards, stitched
    together, equal the full-table model's bit for bit, and so does the merged rank / top-10."""
    import copy
    from gr_amd import dist as D, synth
    items, n, B, d = 1_000_000, 200, 512, 128
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    seqs = synth.sequences(B, n, items, 5000, dev)
    table = synth.table_rows(torch.arange(items + 1, device=dev), d, 7, dev)
    m1, s1 = synth.sasrec_rank_model(items, p, seqs, dev, seed=5)
    full = copy.deepcopy(m1)
    full.item_emb = torch.nn.Embedding(items + 1, d, padding_idx=0).to(dev)
    with torch.no_grad():
        full.item_emb.weight.copy_(table)
    full.item_num = items
    h = full.last_hidden(seqs)
    assert torch.equal(m1.last_hidden(s1), h)
    for world in (2, 8):
        hs = []
        for r in range(world):
            lo, hi = D.shard_range(B, r, world)
            mr, sr = synth.sasrec_rank_model(items, p, seqs[lo:hi], dev, seed=5)
            hs.append(mr.last_hidden(sr))
        assert torch.equal(torch.cat(hs), h), world
        shards = [D.shard_range(items + 1, r, world) for r in range(world)]
        parts = [synth.table_rows(torch.arange(lo, hi, device=dev), d, 7, dev) for lo, hi in shards]
        assert torch.equal(torch.cat(parts), table)
