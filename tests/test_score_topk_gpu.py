"""Fused scoring + top-k + strict counts without logits (gr_score_topk_f32; SURVEY §8(e) C5,
§8f row 2) against the materialised path on the same device.

Bar: bit-exact.  Values and ids equal ``topk(score(h, table))`` after the evaluate.py:27 column-0
mask (the fused kernel shares the scoring kernel's fp32 chain), ties to the lower column, counts
equal ``(logits > thr).sum(1)``.  Shapes cover ragged users / rows, rows < k, exact ties, a
catalog whose logits rise with the column (every item displaces the running top-k: the append
buffers overflow and fold every chunk) and one where they fall."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _reference(h, t, k, id_offset, thr, mask_col0):
    from gr_amd import ops
    lg = ops.score(h, t)
    if mask_col0:
        lg[:, 0] = -1e9
    cnt = (lg > thr[:, None]).sum(1)
    kk = min(k, lg.shape[1])
    o = torch.argsort(lg, dim=1, descending=True, stable=True)[:, :kk]
    v, i = lg.gather(1, o), o + id_offset
    if kk < k:
        v = torch.cat([v, torch.full((v.shape[0], k - kk), float("-inf"), device=v.device)], 1)
        i = torch.cat([i, torch.full((i.shape[0], k - kk), -1, dtype=i.dtype, device=i.device)], 1)
    return v, i, cnt


def _check(h, t, k, id_offset=0, mask_col0=True, seed=0):
    """Both tile sizes of the fused call (32-row tile maxima and 16-row half tiles, option
    topk_half) against the materialised reference, with and without counts."""
    from gr_amd import _lib, ops
    g = torch.Generator(device=h.device).manual_seed(seed)
    thr = torch.randn(h.shape[0], generator=g, device=h.device)
    rv, ri, rc = _reference(h, t, k, id_offset, thr, mask_col0)
    half0 = _lib.get_option("topk_half")
    try:
        for half in (0, 1):
            _lib.set_option("topk_half", half)
            v, i, c = ops.score_topk(h, t, k, id_offset, thresholds=thr, mask_col0=mask_col0)
            assert torch.equal(i, ri), half
            assert torch.equal(v, rv), half
            assert torch.equal(c, rc), half
            v2, i2 = ops.score_topk(h, t, k, id_offset, mask_col0=mask_col0)   # without counts
            assert torch.equal(v2, rv) and torch.equal(i2, ri), half
    finally:
        _lib.set_option("topk_half", half0)


@pytest.mark.parametrize("B,d,rows,k", [(1, 64, 70, 10), (300, 64, 100001, 10), (64, 128, 5000, 16),
                                        (257, 32, 1000, 1), (70, 64, 64, 10), (5, 128, 7, 10),
                                        (513, 128, 20011, 10), (33, 32, 1, 3), (512, 128, 300007, 10),
                                        (100, 32, 150001, 4), (40, 64, 262145, 16),
                                        (200, 16, 707, 10), (65, 16, 100001, 16),   # d 16: SASRec/main.py:12
                                        (512, 128, 1000001, 10),   # C5 full size: 512 users x 1M-item catalog
                                        # larger batches: user blocks that do not divide the resident
                                        # workgroups (2,100 users: 17 blocks), a c5_rank-like shard
                                        (2100, 128, 125000, 10), (4096, 64, 20011, 16)])
def test_score_topk_random(B, d, rows, k, dev):
    g = torch.Generator().manual_seed(B * 7 + d + rows)
    h = torch.randn(B, d, generator=g).to(dev)
    t = torch.randn(rows, d, generator=g).to(dev)
    _check(h, t, k, id_offset=0, mask_col0=True, seed=rows)
    _check(h, t, k, id_offset=12345, mask_col0=False, seed=rows + 1)


def test_score_topk_ties(dev):
    """Duplicated table rows (exact logit ties inside and across lanes, chunks and slices) and a
    constant catalog: the lower column must win every tie."""
    g = torch.Generator().manual_seed(3)
    d, rows = 64, 30001
    t = torch.randn(rows, d, generator=g)
    t[rows // 2:] = t[: rows - rows // 2].clone()
    t[100:164] = t[7]
    h = torch.randn(40, d, generator=g)
    _check(h.to(dev), t.to(dev), 16)
    _check(h.to(dev), torch.ones(4097, d).to(dev), 10)


@pytest.mark.parametrize("direction", [1.0, -1.0])
def test_score_topk_monotone_catalog(direction, dev):
    """Logits strictly monotone in the column for every user: rising = worst case (each new item
    enters every lane's list), falling = best case (nothing after the first chunk)."""
    d, rows, B = 32, 200000, 96
    t = torch.zeros(rows, d)
    t[:, 0] = direction * torch.arange(rows, dtype=torch.float32) / rows
    t[:, 1] = 1.0
    g = torch.Generator().manual_seed(4)
    h = torch.rand(B, d, generator=g) + 0.5
    _check(h.to(dev), t.to(dev), 10)


def test_sharded_fused_equals_full_catalog(dev):
    """Catalog shards scored by the fused kernel (8 sequential shards on one GPU): counts summed
    over shards + 1 and the merged top-k equal the full-catalog rank / top-k bit for bit."""
    from gr_amd import dist as D, ops
    g = torch.Generator().manual_seed(11)
    B, d, rows, k = 200, 128, 40001, 10
    table = torch.randn(rows, d, generator=g).to(dev)
    h = torch.randn(B, d, generator=g).to(dev)
    tg = torch.randint(0, rows, (B,), generator=g).to(dev)
    full = ops.score(h, table)
    ref_rank = ops.rank(full, tg)
    full[:, 0] = -1e9
    o = torch.argsort(full, dim=1, descending=True, stable=True)[:, :k]
    ts = ops.score_pairs(h, table, tg)            # global target logits (column-0 masked)
    cnt = torch.zeros(B, dtype=torch.int64, device=dev)
    vs, is_ = [], []
    for r in range(8):
        lo, hi = D.shard_range(rows, r, 8)
        v, i, c = ops.score_topk(h, table[lo:hi], k, lo, thresholds=ts, mask_col0=(lo == 0))
        cnt += c
        vs.append(v)
        is_.append(i)
    v, i = D.merge_topk(torch.cat(vs, 1), torch.cat(is_, 1), k)
    assert torch.equal(cnt + 1, ref_rank)
    assert torch.equal(i, o) and torch.equal(v, full.gather(1, o))
    # the module-level entry point (world size 1) takes the fused path
    rk, v1, i1 = D.sharded_rank_topk(h, table, 0, tg, k=k)
    assert torch.equal(rk, ref_rank) and torch.equal(i1, o) and torch.equal(v1, v)


@pytest.mark.parametrize("B,C,k", [(1, 80, 10), (4096, 80, 10), (33, 12, 10), (50, 256, 16), (9, 30, 1)])
def test_merge_topk_kernels_equal_torch_merge(B, C, k, dev):
    """gr_merge_topk_f32 / gr_merge_topk_packed (one wave per row) against the torch merge of two
    stable sorts: (value desc, id asc), ids < 0 padding (emitted as (-inf, -1) when fewer than k
    real candidates remain), exact ties across candidate lists (the same value under several ids)."""
    from gr_amd import dist as D, ops
    g = torch.Generator().manual_seed(B + C + k)
    vals = torch.randn(B, C, generator=g)
    vals[:, 3::5] = vals[:, 2::5][:, : vals[:, 3::5].shape[1]]        # equal values, other ids
    ids = torch.randperm(10 * C, generator=g)[:C].repeat(B, 1)
    ids[torch.rand(B, C, generator=g) < (0.4 if C < 2 * k else 0.1)] = -1   # padding
    ref_v, ref_i = D.merge_topk(vals, ids, k)                         # CPU: the torch form
    v, i = ops.merge_topk(vals.to(dev), ids.to(dev), k)
    assert torch.equal(v.cpu(), ref_v) and torch.equal(i.cpu(), ref_i)
    world = 4 if C % 4 == 0 else 1
    kk = C // world
    packed = torch.stack([D._pack(vals[:, r * kk:(r + 1) * kk], ids[:, r * kk:(r + 1) * kk]) for r in range(world)])
    v2, i2 = ops.merge_topk_packed(packed.to(dev), world, kk, k)
    assert torch.equal(v2.cpu(), ref_v) and torch.equal(i2.cpu(), ref_i)


@pytest.mark.parametrize("B,C,k", [(64, 40, 10), (7, 5, 10), (3, 256, 16)])
def test_merge_topk_wide_ids_nan_and_short_rows(B, C, k, dev):
    """ids at and above 2^32 (equal values must still order by the full 64-bit id), NaN
    entries (padding on both paths), fewer real candidates than k (k columns on both paths, padded
    with (-inf, -1)), and the dispatch rules of dist.merge_topk (non-fp32 -> torch form, k < 1 ->
    ValueError)."""
    from gr_amd import dist as D, ops
    g = torch.Generator().manual_seed(B * C + k)
    vals = torch.randn(B, C, generator=g).round(decimals=1)          # many exact value ties
    base = torch.tensor([2 ** 32 - 3, 2 ** 32 - 2, 2 ** 32 - 1, 2 ** 32, 2 ** 32 + 1, 2 ** 40, 5, 0])
    ids = torch.cat([base, torch.randint(0, 2 ** 62, (C,), generator=g)])[:C].repeat(B, 1)
    ids = torch.stack([r[torch.randperm(C, generator=g)] for r in ids])
    vals[:, ::3] = 0.5                                                 # one value under many wide ids
    vals[torch.rand(B, C, generator=g) < 0.1] = float("nan")
    ids[torch.rand(B, C, generator=g) < 0.1] = -1
    ref_v, ref_i = D.merge_topk(vals, ids, k)
    assert ref_v.shape == (B, k)
    v, i = ops.merge_topk(vals.to(dev), ids.to(dev), k)
    assert torch.equal(v.cpu(), ref_v) and torch.equal(i.cpu(), ref_i)
    v3, i3 = D.merge_topk(vals.to(dev), ids.to(dev), k)               # dispatch: the kernel
    assert torch.equal(v3.cpu(), ref_v) and torch.equal(i3.cpu(), ref_i)
    v4, i4 = D.merge_topk(vals.double().to(dev), ids.to(dev), k)      # fp64: the torch form
    assert torch.equal(v4.float().cpu(), ref_v) and torch.equal(i4.cpu(), ref_i)
    with pytest.raises(ValueError):
        D.merge_topk(vals.to(dev), ids.to(dev), 0)


def test_score_topk_rejects_bad_args(dev):
    from gr_amd import ops
    h = torch.randn(4, 64, device=dev)
    t = torch.randn(100, 64, device=dev)
    with pytest.raises(RuntimeError, match="k > 16"):
        ops.score_topk(h, t, 17)
    with pytest.raises(RuntimeError, match="d must be"):
        ops.score_topk(torch.randn(4, 48, device=dev), torch.randn(100, 48, device=dev), 5)


@pytest.mark.parametrize("B,d,rows", [(300, 64, 100001), (2048, 64, 20001), (77, 32, 5003), (1100, 128, 40001),
                                      (129, 128, 9000), (2600, 16, 16001), (50, 16, 707)])
def test_score_layouts_identical(B, d, rows, dev):
    """gr_score_f32 picks its kernel by the logits layout: rows on 128-byte lines (direct stores),
    the reference's contiguous [B, N+1] rows below the Infinity Cache size (direct, cached stores)
    and above it (rotated whole lines; the LDS ring at d 128).  Every layout holds the same bits,
    ragged users / rows included, and nothing is written past a row's columns."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(B + rows)
    h = torch.randn(B, d, generator=g).to(dev)
    t = torch.randn(rows, d, generator=g).to(dev)
    ld = (rows + 31) // 32 * 32
    pad = torch.full((B, ld + 32), 7.0, device=dev)
    ops.score(h, t, out=pad[:, :rows])          # row stride ld + 32: every row on a 128-B line
    assert (pad[:, rows:] == 7.0).all()
    cont = torch.full((B * rows + 64,), 7.0, device=dev)
    view = cont[32:32 + B * rows].view(B, rows)   # contiguous rows, base off the 128-B grid
    ops.score(h, t, out=view)
    assert torch.equal(view, pad[:, :rows])
    assert (cont[:32] == 7.0).all() and (cont[32 + B * rows:] == 7.0).all()


def _gloo_gpu_worker(rank, world, port, data, out, backend="gloo"):
    import os as _os
    import torch.distributed as dist
    _os.environ["MASTER_ADDR"] = "127.0.0.1"
    _os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":   # RCCL, initialised exactly as bench.py does for one rank per GPU
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    from gr_amd import dist as D
    h, table, targets, k = (t.cuda() if torch.is_tensor(t) else t for t in data)
    lo, hi = D.shard_range(table.shape[0], rank, world)
    rk, v, i = D.sharded_rank_topk(h, table[lo:hi].contiguous(), lo, targets, k)   # fused HIP path
    # pipelined over 3 batches: async exchange of batch b overlapped with batch b+1's kernels
    cuts = [0, 40, 41, h.shape[0]]
    res = D.sharded_rank_topk_batches([h[a:b] for a, b in zip(cuts[:-1], cuts[1:])], table[lo:hi].contiguous(),
                                      lo, [targets[a:b] for a, b in zip(cuts[:-1], cuts[1:])], k)
    # the hidden-state gather of the C5 step: every rank's user slice back into the whole batch,
    # balanced (all_gather_into_tensor over RCCL, no padding) and uneven (padded, then sliced)
    sizes = [D.shard_range(h.shape[0], r_, world)[1] - D.shard_range(h.shape[0], r_, world)[0] for r_ in range(world)]
    ulo, uhi = D.shard_range(h.shape[0], rank, world)
    hg = D.all_gather_rows(h[ulo:uhi], sizes=sizes)
    usz = [3 + r_ for r_ in range(world)]
    hu, wk = D.all_gather_rows(h[sum(usz[:rank]):sum(usz[:rank + 1])], sizes=usz, async_op=True)
    if wk is not None:
        wk.wait()
    gathered_ok = torch.equal(hg, h) and torch.equal(hu, h[:sum(usz)])
    # the cross-step form (bench.py's "xstep" exchange): two submits of the whole batch, each
    # result bitwise the serial exchange's
    pipe = D.ShardedRankPipeline(table[lo:hi].contiguous(), lo, k)
    x0 = pipe.submit(h, targets)
    x1 = pipe.submit(h, targets)
    x2 = pipe.flush()
    gathered_ok = gathered_ok and x0 is None and pipe.flush() is None and all(
        torch.equal(a_, b_) for xr in (x1, x2) for a_, b_ in zip(xr, (rk, v, i)))
    out[rank] = (rk.cpu(), v.cpu(), i.cpu(), torch.cat([r_[0] for r_ in res]).cpu(),
                 torch.cat([r_[1] for r_ in res]).cpu(), torch.cat([r_[2] for r_ in res]).cpu(), gathered_ok)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,backend", [(2, "gloo"), (3, "gloo"), (8, "gloo"), (1, "nccl")])
def test_catalog_sharded_fused_multi_rank(world, backend, dev):
    """The catalog-sharded exchange over real ranks (gloo, every rank on this GPU) with the fused
    HIP kernels: every rank returns the full-catalog rank / top-k bit for bit, both through the
    serial exchange, the split one (sharded_rank_topk_batches) and the cross-step one
    (ShardedRankPipeline) -- the three forms bench.py's N > 1 run chooses between;
    world 8 is the C5 node's shard count.  The one-rank RCCL
    case runs every collective of the exchange (a one-rank group still issues them) through the
    "nccl" backend and bench.py's ``device_id`` initialisation: RCCL needs one GPU per rank, so
    this box cannot hold more than one."""
    import socket
    import torch.multiprocessing as mp
    from gr_amd import ops
    g = torch.Generator().manual_seed(21 + world)
    B, d, rows, k = 96, 64, 30011, 10
    table = torch.randn(rows, d, generator=g)
    table[25000] = table[17]            # an exact tie across shards: the lower id wins
    h = torch.randn(B, d, generator=g)
    tg = torch.randint(0, rows, (B,), generator=g)
    tg[0] = 0
    tg[1] = 25000
    full = ops.score(h.to(dev), table.to(dev))
    ref_rank = ops.rank(full, tg.to(dev)).cpu()
    full[:, 0] = -1e9
    o = torch.argsort(full, dim=1, descending=True, stable=True)[:, :k]
    ref_v, ref_i = full.gather(1, o).cpu(), o.cpu()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gloo_gpu_worker, args=(world, port, (h, table, tg, k), out, backend), nprocs=world, join=True)
    for r in range(world):
        rk, v, i, pr, pv, pi, gathered_ok = out[r]
        assert gathered_ok
        assert torch.equal(rk, ref_rank)
        assert torch.equal(i, ref_i) and torch.equal(v, ref_v)
        assert torch.equal(pr, ref_rank) and torch.equal(pi, ref_i) and torch.equal(pv, ref_v)
