"""Multi-rank logic of the catalog-sharded SASRec scoring and the item/user sharding,
exercised with the gloo backend on CPU (world sizes 2 and 3).  The HIP scorer/counter/top-k are
replaced by CPU torch stand-ins with the same semantics; the GPU kernels themselves are covered
by the -m gpu tests."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def cpu_score(h, table):
    return h @ table.t()


def cpu_count(logits, thr):
    return (logits > thr.unsqueeze(1)).sum(1)


def cpu_topk(logits, k, off):
    cols = torch.arange(logits.shape[1]).expand_as(logits)
    o1 = None
    o2 = torch.argsort(logits, dim=1, descending=True, stable=True)
    return logits.gather(1, o2)[:, :k], o2[:, :k] + off


def _worker(rank, world, port, data, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gr_amd.dist as D
    h, table, targets, k = data
    lo, hi = D.shard_range(table.shape[0], rank, world)
    rk, v, i = D.sharded_rank_topk(h, table[lo:hi], lo, targets, k, scorer=cpu_score,
                                   counter=cpu_count, topk_fn=cpu_topk)
    # user-sharded transformer output gathered back (variable shard sizes)
    ulo, uhi = D.shard_range(h.shape[0], rank, world)
    hg = D.all_gather_rows(h[ulo:uhi])
    sizes = [D.shard_range(h.shape[0], r, world)[1] - D.shard_range(h.shape[0], r, world)[0]
             for r in range(world)]
    assert torch.equal(D.all_gather_rows(h[ulo:uhi], sizes=sizes), hg)   # known sizes: no exchange
    # the pipelined form over 3 user batches (exchange of batch b overlapped with batch b+1)
    cuts = [0, 11, 12, B_ := h.shape[0]]
    hs = [h[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    ts = [targets[a:b] for a, b in zip(cuts[:-1], cuts[1:])]
    res = D.sharded_rank_topk_batches(hs, table[lo:hi], lo, ts, k, scorer=cpu_score, counter=cpu_count,
                                      topk_fn=cpu_topk)
    assert len(res) == 3 and B_ == h.shape[0]
    # identical to the sequential per-batch calls (the CPU stand-in matmul is not batch-invariant,
    # so the reference for the pipelined form is the same batches run one after another)
    for (hb, tb), (r1, v1, i1) in zip(zip(hs, ts), res):
        r0, v0, i0 = D.sharded_rank_topk(hb, table[lo:hi], lo, tb, k, scorer=cpu_score, counter=cpu_count,
                                         topk_fn=cpu_topk)
        assert torch.equal(r0, r1) and torch.equal(v0, v1) and torch.equal(i0, i1)
    pr = torch.cat([r_[0] for r_ in res])
    pi = torch.cat([r_[2] for r_ in res])
    # the cross-step form: submit returns the previous batch's result, flush the last one's
    pipe = D.ShardedRankPipeline(table[lo:hi], lo, k, scorer=cpu_score, counter=cpu_count, topk_fn=cpu_topk)
    got = [pipe.submit(hb, tb) for hb, tb in zip(hs, ts)] + [pipe.flush()]
    assert got[0] is None and pipe.flush() is None
    for r_a, r_b in zip(res, got[1:]):
        assert all(torch.equal(x, y) for x, y in zip(r_a, r_b))
    out[rank] = (rk, v, i, hg, (pr, pi))
    dist.barrier()
    dist.destroy_process_group()


def _run(world, data):
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), data, out), nprocs=world, join=True)
    return [out[r] for r in range(world)]


@pytest.mark.parametrize("world", [1, 2, 3])
def test_catalog_sharded_rank_topk_equals_full_catalog(world):
    """world 1: a one-rank group still runs every collective of the exchange (dist._world)."""
    g = torch.Generator().manual_seed(world)
    B, d, rows, k = 37, 16, 1001, 10
    table = torch.randn(rows, d, generator=g)
    table[0] = 0
    # duplicated rows force exact ties across shards (tie -> lower global id)
    table[700] = table[10]
    h = torch.randn(B, d, generator=g)
    targets = torch.randint(0, rows, (B,), generator=g)
    targets[0] = 0          # padding target (evaluate.py: score -1e9)
    targets[1] = 700
    res = _run(world, (h, table, targets, k))
    # single-device reference of evaluate.py:27-32 and a full-catalog top-k
    lg = cpu_score(h, table)
    lg[:, 0] = -1e9
    ts = lg.gather(1, targets.unsqueeze(1))
    ref_rank = (lg > ts).sum(1) + 1
    ref_v, ref_i = cpu_topk(lg, k, 0)
    for rk, v, i, hg, (pr, pi) in res:
        assert torch.equal(rk, ref_rank)
        assert torch.equal(i, ref_i) and torch.equal(v, ref_v)
        assert torch.equal(hg, h)
        assert torch.equal(pr, ref_rank) and torch.equal(pi, ref_i)


def test_merge_topk_tie_and_padding_rules():
    from gr_amd.dist import merge_topk
    vals = torch.tensor([[1.0, 3.0, 3.0, 2.0, 0.0]])
    ids = torch.tensor([[5, 9, 4, 1, -1]])
    v, i = merge_topk(vals, ids, 4)
    assert i.tolist() == [[4, 9, 1, 5]] and v.tolist() == [[3.0, 3.0, 2.0, 1.0]]
    v, i = merge_topk(vals, ids, 5)
    assert i[0, 4].item() == -1
    # fewer candidates than k: k columns, padded (-inf, -1) -- as the GPU kernel emits
    v, i = merge_topk(vals, ids, 8)
    assert v.shape == (1, 8) and i[0, 4:].tolist() == [-1] * 4 and (v[0, 4:] == float("-inf")).all()
    # NaN is padding, never ranked first; wide ids order by all 64 bits
    vals2 = torch.tensor([[float("nan"), 2.0, 2.0, 2.0]])
    ids2 = torch.tensor([[0, 2 ** 33 + 1, 2 ** 33, 2 ** 32 - 1]])
    v, i = merge_topk(vals2, ids2, 4)
    assert i.tolist() == [[2 ** 32 - 1, 2 ** 33, 2 ** 33 + 1, -1]]
    with pytest.raises(ValueError):
        merge_topk(vals, ids, 0)


def test_shard_range_partitions():
    from gr_amd.dist import shard_range
    for n in (0, 1, 7, 100_000, 10_000_000):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[r][1] == parts[r + 1][0] for r in range(w - 1))
            assert max(b - a for a, b in parts) - min(b - a for a, b in parts) <= 1


def test_hr_ndcg_matches_reference_tail():
    from gr_amd.dist import hr_ndcg
    from oracle import metrics_oracle
    ranks = np.array([1, 2, 10, 11, 500, 3, 1])
    assert hr_ndcg(torch.from_numpy(ranks)) == metrics_oracle.hr_ndcg(ranks, 10)


def test_catalog_smaller_than_world_leaves_an_empty_shard():
    """rows = 2 over 3 ranks: one rank holds no catalog rows (the pipelined form indexed
    column 0 of an empty shard).  Ranks and the padded top-k must equal the full-catalog answer."""
    g = torch.Generator().manual_seed(11)
    B, d, rows, k = 23, 8, 2, 4
    table = torch.randn(rows, d, generator=g)
    table[0] = 0
    h = torch.randn(B, d, generator=g)
    targets = torch.randint(0, rows, (B,), generator=g)
    res = _run(3, (h, table, targets, k))
    lg = cpu_score(h, table)
    lg[:, 0] = -1e9
    ref_rank = (lg > lg.gather(1, targets.unsqueeze(1))).sum(1) + 1
    ref_v, ref_i = cpu_topk(lg, rows, 0)
    for rk, v, i, hg, (pr, pi) in res:
        assert torch.equal(rk, ref_rank) and torch.equal(pr, ref_rank)
        assert torch.equal(i[:, :rows], ref_i) and (i[:, rows:] == -1).all()
        # the CPU stand-in matmul is not shape-invariant in its last bits: values to fp32 rounding
        assert torch.allclose(v[:, :rows], ref_v, rtol=1e-6, atol=0) and torch.isinf(v[:, rows:]).all()
        assert torch.equal(pi[:, :rows], ref_i)
