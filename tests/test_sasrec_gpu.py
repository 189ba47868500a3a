"""SASRec forward / predict / rank on the GPU vs the reference's golden vectors.

Bar (north_star): logits within 1e-5 of the row scale (max |logit| of the row: elementwise
relative error is meaningless for logits near 0, SURVEY §7 hard part 4); ranks and HR@10/NDCG@10
equal to the reference.  Ranks are compared exactly for every user whose target logit is
separated from its nearest competitor by more than fp32 noise (fixture ``margin``).
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import metrics_oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5
SAS = ["sas_csv_c1", "sas_syn_c3", "sas_syn_c5", "sas_syn_h2", "sas_syn_d32_h4"]


@pytest.fixture(params=[3, 1, 0], ids=["fused2", "fused", "layerwise"])
def sas_path(request):
    """Run a test through the register-resident fused forward (n <= 64, d <= 64: two waves per
    sequence when n > 32, or one), and through the layer-wise pipeline: all must meet the same bar
    (shapes outside the fused kernel's range run layer-wise either way)."""
    from gr_amd import _lib
    _lib.set_option("sas_fused", request.param)
    yield request.param
    _lib.set_option("sas_fused", 2)


def build(name, dev):
    from gr_amd import SASRec
    sd, out, meta = gl.load(name)
    p = dict(meta["params"], device=str(dev))
    m = SASRec(meta["item_num"], p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    return m.to(dev).eval(), out, meta


@pytest.mark.parametrize("name", SAS)
def test_predict_logits_match_reference(name, dev, sas_path):
    m, out, meta = build(name, dev)
    logits = m.predict(torch.from_numpy(out["seqs"]).to(dev))
    ref = torch.from_numpy(out["logits"])
    got = logits.cpu()
    assert got.shape == ref.shape
    scale = ref.abs().amax(1, keepdim=True)
    err = ((got - ref).abs() / scale).max().item()
    print(f"\n{name}: max row-scaled |dlogit| = {err:.3g}")
    assert err <= TOL


@pytest.mark.parametrize("name", SAS)
def test_ranks_and_hr_ndcg_match_reference(name, dev, sas_path):
    from gr_amd import ops
    m, out, meta = build(name, dev)
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    targets = torch.from_numpy(out["targets"]).to(dev)
    logits = m.predict(seqs)
    ranks = ops.rank(logits, targets).cpu().numpy()
    # evaluate.py:27-32 executed with torch ops on the same GPU logits must agree exactly
    lg = logits.clone()
    lg[:, 0] = -1e9
    ts = lg.gather(1, targets.unsqueeze(1))
    assert np.array_equal(ranks, ((lg > ts).sum(1) + 1).cpu().numpy())
    certified = out["margin"] > 1e-5
    assert np.array_equal(ranks[certified], out["ranks"][certified])
    hr, ndcg = metrics_oracle.hr_ndcg(ranks, 10)
    assert hr == meta["hr10"] and ndcg == pytest.approx(meta["ndcg10"], abs=0, rel=0)


@pytest.mark.parametrize("name", SAS)
def test_forward_matches_reference(name, dev, sas_path):
    m, out, meta = build(name, dev)
    k = out["forward"].shape[0]
    seqs = torch.from_numpy(out["seqs"][:k]).to(dev)
    feats = m.forward(seqs).cpu().numpy()
    assert feats.shape == out["forward"].shape
    assert np.abs(feats - out["forward"]).max() < 5e-5
    # last_hidden (predict's path) runs the final block for position n-1 alone: same math,
    # another fp32 summation order than the full forward's last row
    last = m.last_hidden(seqs).cpu().numpy()
    assert np.abs(last - out["forward"][:, -1, :]).max() < 5e-5
    assert np.abs(last - feats[:, -1, :]).max() < 5e-5


def test_predict_returns_fresh_writable_tensor(dev):
    m, out, meta = build("sas_csv_c1", dev)
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    a = m.predict(seqs)
    a[:, 0] = -1e9      # evaluate.py:27 mutates in place
    b = m.predict(seqs)
    assert not torch.equal(a[:, 0], b[:, 0]) and torch.equal(a[:, 1:], b[:, 1:])


def test_predict_contiguous_by_default(dev):
    """predict returns a contiguous [B, N+1] tensor by default (the reference's matmul layout,
    model.py:107: .view() works), bitwise the row-padded option's values."""
    m, out, meta = build("sas_syn_c3", dev)
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    c = m.predict(seqs)
    try:
        m.contiguous_logits = False
        a = m.predict(seqs)
    finally:
        m.contiguous_logits = True
    assert c.is_contiguous() and c.shape == a.shape and not a.is_contiguous()
    assert torch.equal(a, c)
    assert c.view(-1).numel() == a.numel()


@pytest.mark.parametrize("B,rows,pad,off,d", [(2048, 100001, 0, 0, 64), (700, 60001, 0, 0, 64), (300, 100001, 0, 0, 64),
                                              (1000, 50001, 5, 3, 64), (1500, 40000, 7, 1, 64), (129, 100001, 0, 0, 64),
                                              (2048, 100001, 0, 0, 16), (1000, 50001, 5, 3, 16), (1500, 40000, 7, 1, 32),
                                              (700, 60001, 0, 0, 32)])
def test_score_unaligned_rows_bitwise(dev, B, rows, pad, off, d):
    """Logits rows off the 128-byte grid: the rotated whole-line kernel (> 160 MB of logits) and the
    direct kernel (smaller) against the aligned layout, bit for bit, including a row stride that is
    not rows (pad), a base that is not line-aligned (off), partial user blocks and a partial last
    chunk; every element written exactly once (NaN-filled canvas, guard columns untouched)."""
    from gr_amd import ops
    g = torch.Generator(device=dev).manual_seed(B + rows)
    h = torch.randn(B, d, device=dev, generator=g)
    table = torch.randn(rows, d, device=dev, generator=g)
    ref = ops.logits_buffer(B, rows, dev)
    ops.score(h, table, out=ref)
    canvas = torch.full((B, rows + pad + off), float("nan"), device=dev)
    view = canvas[:, off:off + rows]
    ops.score(h, table, out=view)
    torch.cuda.synchronize()
    assert torch.equal(view, ref)
    if pad + off:
        assert torch.isnan(canvas[:, :off]).all() and torch.isnan(canvas[:, off + rows:]).all()


@pytest.mark.parametrize("name", ["sas_csv_c1", "sas_syn_c3"])
def test_predict_row_padded_layout(name, dev, sas_path):
    """contiguous_logits = False: predict() returns a [B, N+1] view whose rows are 32-float aligned
    (direct-store scoring); the values are bitwise those written into a packed buffer, and
    evaluate.py:27-32 runs on the view."""
    from gr_amd import ops
    m, out, meta = build(name, dev)
    m.contiguous_logits = False
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    targets = torch.from_numpy(out["targets"]).to(dev)
    a = m.predict(seqs)
    rows = meta["item_num"] + 1
    assert a.shape == (len(seqs), rows) and a.stride(1) == 1
    assert a.stride(0) % 32 == 0 and a.data_ptr() % 128 == 0
    packed = torch.empty((len(seqs), rows), device=dev)
    ops.sasrec_predict(m._binding(seqs), seqs, out=packed)
    assert torch.equal(a, packed)
    lg, lp = a.clone(), packed.clone()
    a[:, 0] = -1e9
    packed[:, 0] = -1e9
    ra = (a > a.gather(1, targets.unsqueeze(1))).sum(1) + 1
    rp = (packed > packed.gather(1, targets.unsqueeze(1))).sum(1) + 1
    assert torch.equal(ra, rp) and torch.equal(ops.rank(lg, targets), ra)


def test_deterministic_and_batch_invariant(dev, sas_path):
    m, out, meta = build("sas_syn_c3", dev)
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    a = m.predict(seqs)
    b = torch.cat([m.predict(seqs[i:i + 7]) for i in range(0, len(seqs), 7)])
    assert torch.equal(a, m.predict(seqs))
    assert torch.equal(a, b)


def test_out_of_range_ids_flagged(dev):
    from gr_amd import ops
    m, out, meta = build("sas_csv_c1", dev)
    seqs = torch.from_numpy(out["seqs"]).to(dev).clone()
    seqs[3, -1] = meta["item_num"] + 1
    old = ops.CHECK
    ops.CHECK = True
    try:
        with pytest.raises(IndexError):
            m.predict(seqs)
    finally:
        ops.CHECK = old


def test_sequence_longer_than_max_len_raises(dev):
    m, out, meta = build("sas_csv_c1", dev)
    with pytest.raises(IndexError):
        m.predict(torch.ones((2, 21), dtype=torch.long, device=dev))


@pytest.mark.parametrize("m_,k,n,act,res", [
    (1, 4, 1, "none", False), (130, 36, 70, "relu", False), (257, 768, 256, "relu", False),
    (1000, 64, 192, "none", True), (77, 128, 32, "none", False), (300, 64, 100001, "none", False),
])
def test_linear_vs_fp64(m_, k, n, act, res, dev):
    from gr_amd import ops
    g = torch.Generator().manual_seed(m_ + k + n)
    x = torch.randn(m_, k, generator=g)
    w = torch.randn(n, k, generator=g)
    b = torch.randn(n, generator=g)
    r = torch.randn(m_, n, generator=g) if res else None
    y = ops.linear(x.to(dev), w.to(dev), b.to(dev), act=act,
                   residual=r.to(dev) if res else None).cpu().double()
    ref = x.double() @ w.double().t() + b.double()
    if act == "relu":
        ref = ref.clamp_min(0)
    if res:
        ref = ref + r.double()
    bound = (x.double().abs() @ w.double().abs().t() + b.double().abs()) * 4e-7 * k ** 0.5 + 1e-6
    if res:
        bound = bound + r.double().abs() * 1.2e-7
    assert ((y - ref).abs() <= bound).all()


@pytest.mark.parametrize("m_,n,act", [(102_400, 384, "none"), (64 * 256 + 37, 128, "relu"), (64 * 300 - 1, 256, "none")])
def test_linear_resident_w_equals_tiled(m_, n, act, dev):
    """k = 128, n % 128 == 0 (the C5 block-0 in-projection shape): the persistent kernel with w
    slices resident in registers (option lin_wres) is bitwise the tiled kernel, ragged m included."""
    from gr_amd import _lib, ops
    g = torch.Generator(device=dev).manual_seed(m_ + n)
    x = torch.randn(m_, 128, generator=g, device=dev)
    w = torch.randn(n, 128, generator=g, device=dev) * 0.1
    b = torch.randn(n, generator=g, device=dev)
    try:
        _lib.set_option("lin_wres", 0)
        tiled = ops.linear(x, w, b, act=act)
        _lib.set_option("lin_wres", 1)
        res = ops.linear(x, w, b, act=act)
    finally:
        _lib.set_option("lin_wres", 1)
    assert torch.equal(tiled, res)


@pytest.mark.parametrize("B,blocks", [(37, 2), (515, 2), (9, 1)])
def test_embed_proj_equals_two_kernels(B, blocks, dev):
    """d = 128 block 0 (option emb_proj): embedding gather + LN_a0 + in-projection as one persistent
    kernel with W_in resident in registers is bitwise the embed_ln + gr_linear pair -- full forward
    and last-position predict, ragged row counts; out-of-range ids are still flagged."""
    from gr_amd import _lib, ops, synth
    n, items = 200, 5000
    p = synth.sasrec_params(128, n, blocks, 1, 128, dev)
    m = synth.sasrec_model(items, p, dev, seed=B + blocks)
    seqs = synth.sequences(B, n, items, 7 + B, dev)
    res = {}
    try:
        for opt in (0, 1):
            _lib.set_option("emb_proj", opt)
            res[opt] = (m.forward(seqs), m.predict(seqs))
            bad = seqs.clone()
            bad[B // 2, 5] = items + 3
            old = ops.CHECK
            ops.CHECK = True
            try:
                with pytest.raises(IndexError):
                    m.predict(bad)
            finally:
                ops.CHECK = old
    finally:
        _lib.set_option("emb_proj", 1)
    assert torch.equal(res[1][0], res[0][0])
    assert torch.equal(res[1][1], res[0][1])


@pytest.mark.parametrize("d,heads,n,blocks,B", [(128, 1, 200, 2, 33), (128, 2, 77, 1, 9), (128, 4, 130, 3, 5),
                                                (64, 2, 100, 2, 17), (32, 8, 90, 1, 6)])
def test_tail_h_form_vs_full_block_and_oracle(d, heads, n, blocks, B, dev):
    """A last-position forward's final block (sas_tail_h2_kernel): the one-query tail on LN_a(X)
    with q . K and p . V reassociated through W_k / W_v (no K|V projection) and one pass over H with
    an online softmax per lane group, against the full final block (``forward(...)[:, -1]``, every
    position through the attention kernel) and the CPU oracle: last hidden states within 5e-5,
    predict logits within the row-scaled tolerance; row-tile (d 128) and per-op (d 64 / 32,
    n > 64) paths, 1-8 heads."""
    from gr_amd import synth
    from oracle import sasrec_oracle
    items = 600
    p = synth.sasrec_params(d, n, blocks, heads, 2 * d if d < 128 else 64, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + heads + n)
    seqs = synth.sequences(B, n, items, 5 + n, dev)
    h_h = m.last_hidden(seqs).cpu()
    full = m.forward(seqs)[:, -1, :].cpu()
    got = m.predict(seqs).cpu()
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_f = sasrec_oracle.forward(seqs.cpu(), sd, blocks, heads, 1e-8)
    ref = sasrec_oracle.predict(seqs.cpu(), sd, blocks, heads, 1e-8)
    assert (h_h - ref_f[:, -1, :]).abs().max().item() < 5e-5
    assert (h_h - full).abs().max().item() < 5e-5
    assert (full - ref_f[:, -1, :]).abs().max().item() < 5e-5
    assert ((got - ref).abs() / ref.abs().amax(1, keepdim=True)).max().item() <= TOL


@pytest.mark.parametrize("heads", [1, 2])
def test_tail_reduction_forms_bitwise(heads, dev):
    """sas_tail_h2_kernel's two reduction forms (gr_common.h xsum on the VALU when B <= CUs, ds_bpermute
    above) are the same sums: rows of a 600-sequence call (ds_bpermute form) equal the same rows
    computed in a 100-sequence call (VALU form) bit for bit."""
    from gr_amd import synth
    d, n, items = 128, 200, 3000
    p = synth.sasrec_params(d, n, 2, heads, 64, dev)
    m = synth.sasrec_model(items, p, dev, seed=91 + heads)
    seqs = synth.sequences(600, n, items, 97, dev)
    big = m.last_hidden(seqs)
    small = m.last_hidden(seqs[200:300].contiguous())
    assert torch.equal(big[200:300], small)


@pytest.mark.parametrize("d,heads,n,blocks,B", [(128, 1, 200, 2, 37), (128, 2, 130, 2, 9), (64, 1, 100, 2, 17),
                                                (64, 2, 77, 1, 5), (128, 1, 33, 1, 3), (128, 1, 200, 2, 1500),
                                                (128, 2, 97, 3, 40), (128, 1, 256, 1, 70), (64, 1, 20, 1, 2000)])
def test_attn_persist_vs_oracle(d, heads, n, blocks, B, dev):
    """Layer-wise causal attention at head width 64 / 128 (hd 128: attn_k16_kernel, 32-query tiles over
    16-key steps at two waves per SIMD, and with option attn_k16 0 attn_persist_kernel, 32 x 32 steps
    at one wave per SIMD; both persistent grids over static longest-first item lists; B 1500: ~14
    items per wave; n 20 at B 2000: one query tile, more items than waves) through the
    full forward, against the CPU oracle; the row-tile (d 128) and per-op paths agree within the
    oracle tolerance, and every row is batch-invariant (a sub-batch gives the same bits)."""
    from gr_amd import _lib, synth
    from oracle import sasrec_oracle
    items = 500
    p = synth.sasrec_params(d, n, blocks, heads, 64, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + n)
    seqs = synth.sequences(B, n, items, 3 + n, dev)
    pick = torch.arange(0, B, max(1, B // 64), device=dev)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_f = sasrec_oracle.forward(seqs[pick].cpu(), sd, blocks, heads, 1e-8)
    outs = {}
    try:
        _lib.set_option("sas_fused", 0)
        for k16 in (1, 0):   # hd 128: attn_k16_kernel (16-key steps) by default, then the 32 x 32 steps
            _lib.set_option("attn_k16", k16)
            f = m.forward(seqs)
            sub = m.forward(seqs[:3])
            assert torch.equal(sub, f[:3])
            assert (f[pick].cpu() - ref_f).abs().max().item() < 5e-5
            outs[k16] = f
    finally:
        _lib.set_option("sas_fused", 2)
        _lib.set_option("attn_k16", 1)
    # the two forms are different fp32 chains of the same attention
    assert (outs[1] - outs[0]).abs().max().item() < 2e-5


@pytest.mark.parametrize("d,heads,n,blocks,B", [(64, 1, 50, 2, 300), (64, 2, 64, 2, 33), (32, 4, 20, 1, 17),
                                                (48, 2, 37, 3, 9), (64, 8, 63, 2, 5), (32, 1, 1, 2, 11),
                                                (16, 2, 2, 1, 4), (16, 1, 20, 2, 64)])
def test_fused_tail_h_vs_full_block_and_oracle(d, heads, n, blocks, B, dev):
    """The fused d <= 64 forward's final block for the last position in the H form (no K / V of the
    n tokens) against the fused full forward's last position and the CPU oracle: last hidden state
    within 5e-5, predict logits within the row-scaled tolerance (1-8 heads, padded widths d 16 / 48:
    the padded features of q' are zeroed)."""
    from gr_amd import _lib, synth
    from oracle import sasrec_oracle
    items = 400
    p = synth.sasrec_params(d, n, blocks, heads, 2 * d, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + heads + n)
    seqs = synth.sequences(B, n, items, 7 + n, dev)
    _lib.set_option("sas_fused", 3)
    try:
        h_h = m.last_hidden(seqs).cpu()
        full = m.forward(seqs)[:, -1, :].cpu()
        got = m.predict(seqs).cpu()
    finally:
        _lib.set_option("sas_fused", 2)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_f = sasrec_oracle.forward(seqs.cpu(), sd, blocks, heads, 1e-8)
    ref = sasrec_oracle.predict(seqs.cpu(), sd, blocks, heads, 1e-8)
    assert torch.isfinite(h_h).all()
    assert (h_h - ref_f[:, -1, :]).abs().max().item() < 5e-5
    assert (h_h - full).abs().max().item() < 5e-5
    assert ((got - ref).abs() / ref.abs().amax(1, keepdim=True)).max().item() <= TOL


def test_score_matches_linear_and_rank_consistency(dev):
    """Fused-rank hard part 3: every logit sees the same fp32 fma chain, so the target's score
    recomputed on any tile equals its entry in the logits (strict '>' never counts the target)."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(3)
    h = torch.randn(33, 64, generator=g).to(dev)
    table = torch.randn(5001, 64, generator=g).to(dev)
    lg = ops.score(h, table)
    perm = torch.randperm(5001, generator=g).to(dev)
    lg2 = ops.score(h, table[perm])
    assert torch.equal(lg[:, perm], lg2)
    t = torch.randint(1, 5001, (33,), generator=g).to(dev)
    ranks = ops.rank(lg, t)
    assert (ranks >= 1).all()


def test_count_gt_and_topk_kernels(dev):
    """gr_count_gt_f32 / gr_topk_f32 vs torch on the same device logits (ties included)."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(5)
    lg = torch.randn(65, 3001, generator=g)
    lg[:, 1234] = lg[:, 17]          # exact ties: the lower column must win
    lg[3, :] = 1.0                   # a constant row
    lgd = lg.to(dev)
    thr = lg[torch.arange(65), torch.randint(0, 3001, (65,), generator=g)]
    assert torch.equal(ops.count_gt(lgd, thr.to(dev)).cpu(), (lg > thr[:, None]).sum(1))
    for k in (1, 10, 16, 40):
        v, i = ops.topk(lgd, k, id_offset=1000)
        o = torch.argsort(lg, dim=1, descending=True, stable=True)[:, :k]
        assert torch.equal(i.cpu(), o + 1000)
        assert torch.equal(v.cpu(), lg.gather(1, o))
    v, i = ops.topk(lgd[:, :5], 10)
    assert (i.cpu()[:, 5:] == -1).all()


def test_sharded_scoring_on_one_gpu_equals_full_catalog(dev):
    """Catalog-sharded rank/top-k simulated as 8 sequential shards on one GPU with the
    HIP kernels: the strict-'>' counts summed over shards and the merged top-k equal the
    full-catalog result bit for bit."""
    from gr_amd import dist as D, ops
    g = torch.Generator().manual_seed(9)
    B, d, rows, k = 64, 128, 8001, 10
    table = torch.randn(rows, d, generator=g).to(dev)
    h = torch.randn(B, d, generator=g).to(dev)
    t = torch.randint(1, rows, (B,), generator=g).to(dev)
    full = ops.score(h, table)
    ref_rank = ops.rank(full, t)
    full[:, 0] = -1e9
    ref_v, ref_i = ops.topk(full, k)
    cnt = torch.zeros(B, dtype=torch.int64, device=dev)
    ts = torch.zeros(B, device=dev)
    vs, is_ = [], []
    shards = [D.shard_range(rows, r, 8) for r in range(8)]
    parts = [ops.score(h, table[lo:hi]) for lo, hi in shards]
    for (lo, hi), lg in zip(shards, parts):
        if lo == 0:
            lg[:, 0] = -1e9
        own = (t >= lo) & (t < hi)
        ts += torch.where(own, lg.gather(1, (t - lo).clamp(0, hi - lo - 1).unsqueeze(1)).squeeze(1),
                          torch.zeros_like(ts))
    for (lo, hi), lg in zip(shards, parts):
        cnt += ops.count_gt(lg, ts)
        v, i = ops.topk(lg, k, lo)
        vs.append(v)
        is_.append(i)
    v, i = D.merge_topk(torch.cat(vs, 1), torch.cat(is_, 1), k)
    assert torch.equal(cnt + 1, ref_rank)
    assert torch.equal(i, ref_i) and torch.equal(v, ref_v)


@pytest.mark.parametrize("B,d,rows", [(1, 64, 33), (300, 64, 100001), (64, 128, 5000), (257, 32, 1000),
                                      (5, 16, 77), (300, 16, 100001), (3, 48, 90)])
def test_score_kernel_vs_fp64(B, d, rows, dev):
    """gr_score_f32 (dedicated streaming kernels for d in {16, 32, 64, 128}, the linear GEMM
    otherwise) against an fp64 reference, ragged B / rows included."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(B + d + rows)
    h = torch.randn(B, d, generator=g)
    t = torch.randn(rows, d, generator=g)
    y = ops.score(h.to(dev), t.to(dev)).cpu().double()
    ref = h.double() @ t.double().t()
    bound = (h.double().abs() @ t.double().abs().t()) * 4e-7 * d ** 0.5 + 1e-6
    assert ((y - ref).abs() <= bound).all()


@pytest.mark.parametrize("d,heads,mlp,n,blocks,B", [
    (64, 1, 64, 50, 2, 37), (64, 1, 64, 64, 2, 5), (64, 1, 64, 1, 2, 9), (32, 1, 32, 32, 1, 6),
    (32, 1, 32, 33, 3, 7), (16, 1, 64, 20, 2, 3), (48, 2, 96, 40, 2, 11), (64, 8, 128, 17, 4, 4),
    (40, 5, 20, 64, 1, 13), (64, 2, 64, 50, 8, 2),
])
def test_fused_forward_vs_oracle(d, heads, mlp, n, blocks, B, dev):
    """The fused kernel across its whole shape range (token / feature / mlp tiles, exact and padded
    widths, narrow heads, n = 1, tile boundaries) against the CPU oracle, forward and predict."""
    from gr_amd import _lib, synth
    from oracle import sasrec_oracle
    items = 500
    p = synth.sasrec_params(d, n, blocks, heads, mlp, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + n + blocks)
    seqs = synth.sequences(B, n, items, 3 + n, dev)
    sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
    ref_f = sasrec_oracle.forward(seqs.cpu(), sd, blocks, heads, 1e-8)
    ref = sasrec_oracle.predict(seqs.cpu(), sd, blocks, heads, 1e-8)
    try:
        for opt in (1, 3):   # one wave per sequence; two when n > 32
            _lib.set_option("sas_fused", opt)
            got_f = m.forward(seqs).cpu()
            assert (got_f - ref_f).abs().max().item() < 5e-5
            got = m.predict(seqs).cpu()
            err = ((got - ref).abs() / ref.abs().amax(1, keepdim=True)).max().item()
            assert err <= TOL, err
            assert (m.last_hidden(seqs).cpu() - ref_f[:, -1, :]).abs().max().item() < 5e-5
    finally:
        _lib.set_option("sas_fused", 2)


@pytest.mark.parametrize("d,heads,mlp,n,blocks,B", [
    (64, 1, 64, 50, 2, 37), (64, 1, 64, 64, 2, 5), (32, 1, 32, 33, 3, 7), (48, 2, 96, 40, 2, 11),
    (40, 5, 20, 64, 1, 13), (64, 2, 64, 50, 8, 2), (64, 8, 128, 63, 2, 5), (16, 2, 32, 47, 2, 6),
    (64, 1, 64, 50, 2, 300),
])
def test_fused_two_waves_equal_one_wave(d, heads, mlp, n, blocks, B, dev):
    """sas_fused = 3 (two waves per sequence, wave w owning token tile w, tile 0's K / V handed
    to wave 1 through LDS) runs the one-wave kernel's instruction sequence per token tile: forward,
    last_hidden and predict bitwise equal to sas_fused = 1 (32 < n <= 64, exact and padded widths,
    1-8 heads, 1-8 blocks).  The default (2) picks one of the two by batch size."""
    from gr_amd import _lib, synth
    items = 500
    p = synth.sasrec_params(d, n, blocks, heads, mlp, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + n + blocks + 1)
    seqs = synth.sequences(B, n, items, 5 + n, dev)
    res = {}
    try:
        for opt in (1, 3):
            _lib.set_option("sas_fused", opt)
            res[opt] = (m.forward(seqs), m.last_hidden(seqs), m.predict(seqs))
    finally:
        _lib.set_option("sas_fused", 2)
    for a_, b_ in zip(res[1], res[3]):
        assert torch.isfinite(a_).all()
        assert torch.equal(a_, b_)


@pytest.mark.parametrize("B,d,rows", [(128, 64, 100001), (5, 16, 707), (300, 32, 20000), (64, 128, 125000)])
def test_score_count_workspace_form(B, d, rows, dev):
    """gr_score_count_gt_ws_f32 (counts spread over 16 zeroed copies, then summed) equals the
    direct-atomic form and a torch count over the materialised logits, and leaves its workspace zero."""
    import ctypes
    from gr_amd import _lib as L, ops
    g = torch.Generator(device=dev).manual_seed(B + d)
    h = torch.randn(B, d, generator=g, device=dev) * 0.3
    t = torch.randn(rows, d, generator=g, device=dev)
    th = ops.score_pairs(h, t, torch.randint(0, rows, (B,), generator=g, device=dev), mask_col0=True)
    nb = L.lib().gr_score_count_workspace_bytes(B)
    ws = torch.zeros(nb, dtype=torch.uint8, device=dev)
    a = torch.empty(B, dtype=torch.int64, device=dev)
    b = torch.empty(B, dtype=torch.int64, device=dev)
    st = L.stream_of(dev)
    for _ in range(2):   # the second call relies on the first leaving the workspace zero
        L.check(L.lib().gr_score_count_gt_ws_f32(L.ptr(h), B, d, L.ptr(t), rows, L.ptr(th), 1, L.ptr(a), L.ptr(ws),
                                                 ctypes.c_size_t(nb), st), "ws")
    L.check(L.lib().gr_score_count_gt_f32(L.ptr(h), B, d, L.ptr(t), rows, L.ptr(th), 1, L.ptr(b), st), "direct")
    lg = ops.score(h, t)
    lg[:, 0] = -1e9
    ref = (lg > th[:, None]).sum(1)
    assert torch.equal(a, b) and torch.equal(a, ref)
    assert int(ws.sum().item()) == 0


@pytest.mark.parametrize("B,cols,ld", [(7, 100001, 100001), (33, 250000, 250003), (300, 5, 5), (2, 1, 1)])
def test_segmented_topk_count_vs_torch(B, cols, ld, dev):
    """Segmented top-k / count kernels on long, misaligned (odd stride) rows, single fused pass."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(B + cols)
    base = torch.randn(B, ld, generator=g)
    base[:, cols // 3] = base[:, cols // 2]          # ties across segments: lower column wins
    lg = base[:, :cols]
    lgd = base.to(dev)[:, :cols]
    thr = lg[torch.arange(B), torch.randint(0, cols, (B,), generator=g)]
    k = min(10, cols)
    v, i, c = ops.topk(lgd, k, id_offset=7, thresholds=thr.to(dev))
    o = torch.argsort(lg, dim=1, descending=True, stable=True)[:, :k]
    assert torch.equal(i.cpu(), o + 7) and torch.equal(v.cpu(), lg.gather(1, o))
    assert torch.equal(c.cpu(), (lg > thr[:, None]).sum(1))
    assert torch.equal(ops.count_gt(lgd, thr.to(dev)).cpu(), (lg > thr[:, None]).sum(1))


def test_binding_cache_sees_weight_changes(dev):
    """The cached SasrecBinding follows in-place updates and storage swaps."""
    m, out, meta = build("sas_syn_c3", dev)
    seqs = torch.from_numpy(out["seqs"][:16]).to(dev)
    a = m.predict(seqs).clone()
    with torch.no_grad():
        m.last_layernorm.weight.mul_(2.0)                    # in place
    b = m.predict(seqs).clone()
    assert not torch.equal(a, b)
    m.last_layernorm.weight.data = m.last_layernorm.weight.data / 2.0   # new storage
    c = m.predict(seqs)
    assert torch.equal(a, c)


@pytest.mark.parametrize("rowtile", [1, 0], ids=["rowtile", "per_op"])
@pytest.mark.parametrize("heads,mlp,n,blocks,B", [(1, 64, 200, 2, 6), (2, 32, 77, 3, 5), (4, 128, 33, 1, 4),
                                                  (1, 64, 1, 2, 3), (1, 128, 65, 2, 70), (1, 64, 208, 1, 3),
                                                  (2, 64, 209, 2, 3)])
def test_d128_layerwise_paths_vs_oracle(heads, mlp, n, blocks, B, rowtile, dev):
    """d = 128 (the C5 width): the row-tile fused forward (embed+LN, post-attention row tiles, the
    last-position tail) and the one-kernel-per-op forward, against the CPU oracle; forward (all
    positions), last_hidden and predict; n = 208 / 209 with 16 lane groups of 13 keys at the
    edge."""
    from gr_amd import _lib, synth
    from oracle import sasrec_oracle
    _lib.set_option("sas_rowtile", rowtile)
    try:
        items = 700
        p = synth.sasrec_params(128, n, blocks, heads, mlp, dev)
        m = synth.sasrec_model(items, p, dev, seed=n + blocks)
        seqs = synth.sequences(B, n, items, 11 + n, dev)
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items()}
        ref_f = sasrec_oracle.forward(seqs.cpu(), sd, blocks, heads, 1e-8)
        got_f = m.forward(seqs).cpu()
        assert (got_f - ref_f).abs().max().item() < 5e-5
        assert (m.last_hidden(seqs).cpu() - ref_f[:, -1, :]).abs().max().item() < 5e-5
        ref = sasrec_oracle.predict(seqs.cpu(), sd, blocks, heads, 1e-8)
        got = m.predict(seqs).cpu()
        assert ((got - ref).abs() / ref.abs().amax(1, keepdim=True)).max().item() <= TOL
    finally:
        _lib.set_option("sas_rowtile", 1)
