"""Multi-GPU layer: one process per GPU, ``torch.distributed`` (RCCL over xGMI) — SURVEY §8(e).

The reference is single-device ("device": "cuda:0", RQ-VAE/main.py:34, SASRec/main.py:8).  Both
hot paths are data-parallel:

* RQ encode: items shard across ranks (``shard_range``); no collective on the data path.
* SASRec C3: users shard across ranks; no collective.
* SASRec C5 (1M-item catalog): the *catalog* shards.  ``sharded_rank_topk`` scores every user
  against the local rows, then exchanges only per-user scalars and k candidates:
    1. the owner of each target contributes the target's logit (zeros elsewhere) to an
       all-reduce(sum) — the logit comes out of the same scoring kernel, so its bits equal the
       full-catalog value and the strict '>' never counts the target itself (SURVEY §7 part 3);
    2. local strict-'>' counts -> all-reduce(sum) -> global rank (SASRec/evaluate.py:27-32);
    3. local top-k (value, global id) -> all-gather -> deterministic merge (value desc, id asc).
  Messages are B*(8 + 8 + 12k) bytes per rank: latency-bound over xGMI, never bandwidth-bound.

The scorer / counter / top-k callables default to the HIP kernels (``ops``); they are parameters
only so that the collective logic can be exercised with the gloo backend on CPU in tests.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous, balanced [lo, hi) slice of n units for ``rank`` of ``world``."""
    return n * rank // world, n * (rank + 1) // world


def all_gather_rows(t, group=None, sizes=None, async_op=False):
    """Concatenate a [n_r, ...] tensor over ranks (n_r may differ by rank).  ``sizes`` (every
    rank's n_r, e.g. from ``shard_range``) skips the size exchange and its host synchronisation.

    Over RCCL the rows land in ONE [world * max(n_r), ...] tensor (``all_gather_into_tensor``: one
    collective, no per-rank list, no concatenation when every rank holds the same count -- the C5
    bench's case); other backends (gloo) gather a list.  ``async_op``: returns ``(result, work)``
    with ``result`` valid after ``work.wait()`` (RCCL only; elsewhere the gather has completed)."""
    world = dist.get_world_size(group)
    if sizes is None:
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        sz = [torch.zeros_like(n) for _ in range(world)]
        dist.all_gather(sz, n, group=group)
        sizes = [int(s.item()) for s in sz]
    if sizes[dist.get_rank(group)] != t.shape[0]:
        raise ValueError(f"all_gather_rows: this rank holds {t.shape[0]} rows, sizes say "
                         f"{sizes[dist.get_rank(group)]}")
    m = max(sizes)
    buf = t.contiguous()
    if t.shape[0] < m:
        buf = torch.cat([buf, torch.zeros((m - t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)])
    if t.is_cuda and dist.get_backend(group) == "nccl":
        out = torch.empty((world * m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        work = dist.all_gather_into_tensor(out, buf, group=group, async_op=async_op)
        if any(s != m for s in sizes):
            if async_op:
                work.wait()
                work = None
            out = torch.cat([out[r * m:r * m + s] for r, s in enumerate(sizes)])
        return (out, work) if async_op else out
    parts = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    out = torch.cat([o[:s] for o, s in zip(parts, sizes)])
    return (out, None) if async_op else out


def merge_topk(vals, ids, k):
    """Top-k of candidate lists [B, C] (values, global ids): value descending, ties to the lower id.
    Padding: an entry whose id is < 0 or whose value is NaN (a NaN never ranks).  The result has
    exactly ``k`` columns; when fewer than ``k`` real candidates exist the rest are (-inf, -1).
    ``k`` < 1 raises ValueError.  fp32 CUDA rows of <= 256 candidates: one wave per row
    (ops.merge_topk, gr_merge_topk_f32); everything else (CPU tensors -- the gloo tests -- other
    dtypes, wider rows): the torch form below (two stable sorts), with the same result."""
    if k < 1:
        raise ValueError(f"merge_topk: k must be >= 1, got {k}")
    if vals.is_cuda and vals.dtype == torch.float32 and vals.shape[1] <= 256:
        from . import ops
        return ops.merge_topk(vals, ids, k)
    pad = (ids < 0) | torch.isnan(vals)
    v = torch.where(pad, torch.full_like(vals, float("-inf")), vals)
    big = torch.iinfo(torch.int64).max
    i = torch.where(pad, torch.full_like(ids, big), ids.to(torch.int64))
    if v.shape[1] < k:                                             # fewer candidates than k: pad
        extra = k - v.shape[1]
        v = torch.cat([v, torch.full((v.shape[0], extra), float("-inf"), dtype=v.dtype, device=v.device)], 1)
        i = torch.cat([i, torch.full((i.shape[0], extra), big, dtype=i.dtype, device=i.device)], 1)
    o1 = torch.argsort(i, dim=1, descending=False, stable=True)                    # secondary key: id ascending
    v1, i1 = v.gather(1, o1), i.gather(1, o1)
    o2 = torch.argsort(v1, dim=1, descending=True, stable=True)  # primary key: value descending
    vk, ik = v1.gather(1, o2)[:, :k], i1.gather(1, o2)[:, :k]
    return vk, torch.where(ik == big, torch.full_like(ik, -1), ik)


def _world(group):
    """World size of ``group`` when a process group is initialised, else 0 (no exchange at all).
    A one-rank group still runs every collective, so a single-GPU job launched under
    torch.distributed exercises the same RCCL calls as the 8-GPU one."""
    return dist.get_world_size(group) if dist.is_initialized() else 0


def _default_ops():
    from . import ops
    return ops.score, ops.count_gt, ops.topk


@torch.no_grad()
def sharded_rank_topk(h, table_shard, row_offset, targets, k=10, group=None, mask_row0=True,
                      scorer=None, counter=None, topk_fn=None):
    """Catalog-sharded scoring: every rank holds ``table_shard`` = rows [row_offset, ...) of the
    item table and the same ``h`` [B, d] / global ``targets`` [B].  Returns (rank [B] int64,
    top values [B, k], top ids [B, k]) identical on every rank."""
    world = _world(group)
    rows = table_shard.shape[0]
    if (scorer is None and counter is None and topk_fn is None and h.is_cuda and rows > 0
            and 1 <= k <= 16 and h.shape[1] in (16, 32, 64, 128)):
        return _sharded_rank_topk_fused(h, table_shard, row_offset, targets, k, group, mask_row0, world)
    s_fn, c_fn, t_fn = _default_ops()
    scorer, counter, topk_fn = scorer or s_fn, counter or c_fn, topk_fn or t_fn
    logits = scorer(h, table_shard)
    rows = logits.shape[1]
    if mask_row0 and row_offset == 0 and rows > 0:
        logits[:, 0] = -1e9                                  # evaluate.py:27
    t = targets.reshape(-1).to(torch.int64)
    own = (t >= row_offset) & (t < row_offset + rows)
    local = torch.where(own, t - row_offset, torch.zeros_like(t))
    zero = torch.zeros_like(t, dtype=logits.dtype)
    ts = torch.where(own, logits.gather(1, local.unsqueeze(1)).squeeze(1), zero) if rows > 0 else zero
    if world:
        dist.all_reduce(ts, op=dist.ReduceOp.SUM, group=group)
    kk = min(k, rows) if rows > 0 else 0
    if kk > 0 and topk_fn is t_fn and counter is c_fn:
        v, i, cnt = topk_fn(logits, kk, row_offset, thresholds=ts)   # one pass: top-k + counts
    else:
        cnt = counter(logits, ts)
        if kk > 0:
            v, i = topk_fn(logits, kk, row_offset)
        else:
            v = torch.empty((logits.shape[0], 0), dtype=logits.dtype, device=logits.device)
            i = torch.empty((logits.shape[0], 0), dtype=torch.int64, device=logits.device)
    if kk < k:
        pad = k - kk
        v = torch.cat([v, torch.full((v.shape[0], pad), float("-inf"), dtype=v.dtype, device=v.device)], 1)
        i = torch.cat([i, torch.full((i.shape[0], pad), -1, dtype=i.dtype, device=i.device)], 1)
    return _exchange(cnt, v, i, k, group, world)


def _pack(v, i):
    """[ids | value bits] per user as int64 words: the one tensor the candidates travel in."""
    return torch.cat([i, v.contiguous().view(torch.int32).to(torch.int64)], 1)


def _gather_packed(packed, world, group, async_op=False):
    """All-gather of the packed candidates: into one [world, B, 2 kk] tensor over RCCL (the merge
    kernel reads it as is), a list of per-rank tensors otherwise (gloo)."""
    if packed.is_cuda and dist.get_backend(group) == "nccl":
        out = torch.empty((world,) + tuple(packed.shape), dtype=packed.dtype, device=packed.device)
        work = dist.all_gather_into_tensor(out.view(-1, packed.shape[1]), packed, group=group, async_op=async_op)
        return out, work
    parts = [torch.empty_like(packed) for _ in range(world)]
    return parts, dist.all_gather(parts, packed, group=group, async_op=async_op)


def _merge_gathered(gathered, world, kk, k):
    if not torch.is_tensor(gathered) and gathered[0].is_cuda:   # gloo on device tensors (rehearsal)
        gathered = torch.stack(gathered)
    if torch.is_tensor(gathered):   # [world, B, 2 kk] on the GPU: one kernel unpacks and merges
        from . import ops
        return ops.merge_topk_packed(gathered, world, kk, k)
    ids = torch.cat([p_[:, :kk] for p_ in gathered], 1)
    vals = torch.cat([p_[:, kk:].to(torch.int32).view(torch.float32) for p_ in gathered], 1)
    return merge_topk(vals, ids, k)


def _exchange(cnt, v, i, k, group, world):
    """Steps 2-3 of the module docstring: global counts and the merged top-k.  The (value, id)
    candidates travel as ONE int64 all-gather: [ids | value bits] per user."""
    if world:
        dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=group)
        kk = v.shape[1]
        gathered, _ = _gather_packed(_pack(v, i), world, group)
        v, i = _merge_gathered(gathered, world, kk, k)
    return cnt + 1, v, i


def _sharded_rank_topk_fused(h, table_shard, row_offset, targets, k, group, mask_row0, world):
    """The same exchange with the shard's logits never materialised: the target logit comes from
    ``score_pairs`` and the counts + local top-k from one ``score_topk`` pass over the shard
    (bitwise the values of the unfused path: all three kernels share one fp32 chain)."""
    from . import ops
    rows = table_shard.shape[0]
    m0 = bool(mask_row0 and row_offset == 0)
    t = targets.reshape(-1).to(torch.int64)
    own = (t >= row_offset) & (t < row_offset + rows)
    local = torch.where(own, t - row_offset, torch.zeros_like(t))
    ts = torch.where(own, ops.score_pairs(h, table_shard, local, mask_col0=m0),
                     torch.zeros(t.shape, dtype=torch.float32, device=h.device))
    if world:
        dist.all_reduce(ts, op=dist.ReduceOp.SUM, group=group)
    kk = min(k, rows)
    v, i, cnt = ops.score_topk(h, table_shard, kk, row_offset, thresholds=ts, mask_col0=m0)
    if kk < k:
        pad = k - kk
        v = torch.cat([v, torch.full((v.shape[0], pad), float("-inf"), dtype=v.dtype, device=v.device)], 1)
        i = torch.cat([i, torch.full((i.shape[0], pad), -1, dtype=i.dtype, device=i.device)], 1)
    return _exchange(cnt, v, i, k, group, world)


class _RankStages:
    """The three stages of one batch's catalog-sharded rank + top-k with every collective issued
    ``async_op=True`` (RCCL runs it on its own stream after the work it depends on; the host never
    blocks): ``targets_start`` (the owner's target logits -> all-reduce), ``score_start`` (local
    strict counts + top-k -> count all-reduce + candidate all-gather), ``finish`` (wait, merge).
    Shared by ``sharded_rank_topk_batches`` and ``ShardedRankPipeline``."""

    def __init__(self, table_shard, row_offset, k, group, mask_row0, scorer, counter, topk_fn, h0):
        self.table, self.lo, self.k, self.group = table_shard, row_offset, k, group
        self.world = _world(group)
        self.rows = rows = table_shard.shape[0]
        self.fused = (scorer is None and counter is None and topk_fn is None and h0.is_cuda and rows > 0
                      and 1 <= k <= 16 and h0.shape[1] in (16, 32, 64, 128))
        if not self.fused:
            s_fn, c_fn, t_fn = _default_ops()
            scorer, counter, topk_fn = scorer or s_fn, counter or c_fn, topk_fn or t_fn
        self.scorer, self.counter, self.topk_fn = scorer, counter, topk_fn
        self.m0 = bool(mask_row0 and row_offset == 0)
        self.kk = min(k, rows)

    def targets_start(self, h, t):
        t = t.reshape(-1).to(torch.int64)
        rows, lo = self.rows, self.lo
        own = (t >= lo) & (t < lo + rows)
        local = torch.where(own, t - lo, torch.zeros_like(t))
        logits = None
        if self.fused:
            from . import ops
            tl = ops.score_pairs(h, self.table, local, mask_col0=self.m0)
        else:
            logits = self.scorer(h, self.table)
            if self.m0 and rows > 0:
                logits[:, 0] = -1e9                                  # evaluate.py:27
            tl = (logits.gather(1, local.unsqueeze(1)).squeeze(1) if rows > 0   # an empty shard owns
                  else torch.zeros(t.shape, dtype=logits.dtype, device=logits.device))   # no target
        ts = torch.where(own, tl, torch.zeros(t.shape, dtype=tl.dtype, device=tl.device))
        return ts, logits, dist.all_reduce(ts, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def score_start(self, h, st):
        ts, logits, work = st
        work.wait()
        k, kk = self.k, self.kk
        if self.fused:
            from . import ops
            v, i, cnt = ops.score_topk(h, self.table, kk, self.lo, thresholds=ts, mask_col0=self.m0)
        elif kk > 0:
            cnt = self.counter(logits, ts)
            v, i = self.topk_fn(logits, kk, self.lo)
        else:   # empty shard (a catalog smaller than the world): no count, no candidate
            cnt = torch.zeros(logits.shape[0], dtype=torch.int64, device=logits.device)
            v = torch.empty((logits.shape[0], 0), dtype=logits.dtype, device=logits.device)
            i = torch.empty((logits.shape[0], 0), dtype=torch.int64, device=logits.device)
        if kk < k:
            v = torch.cat([v, torch.full((v.shape[0], k - kk), float("-inf"), dtype=v.dtype, device=v.device)], 1)
            i = torch.cat([i, torch.full((i.shape[0], k - kk), -1, dtype=i.dtype, device=i.device)], 1)
        w1 = dist.all_reduce(cnt, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        gathered, w2 = _gather_packed(_pack(v, i), self.world, self.group, async_op=True)
        return cnt, gathered, w1, w2

    def finish(self, sc):
        cnt, gathered, w1, w2 = sc
        w1.wait()
        w2.wait()
        v, i = _merge_gathered(gathered, self.world, self.k, self.k)
        return cnt + 1, v, i


@torch.no_grad()
def sharded_rank_topk_batches(hs, table_shard, row_offset, targets, k=10, group=None, mask_row0=True,
                              scorer=None, counter=None, topk_fn=None):
    """``[sharded_rank_topk(h, ...) for h in hs]`` with the exchange of each batch overlapped with
    the scoring of the next: the collectives are issued ``async_op=True`` (RCCL runs
    them on its own stream after the scoring they depend on; the host never blocks), in the order
      targets(b+1) -> scoring(b) -> [exchange(b) | scoring(b+1)] -> merge(b) ...
    so the target-logit all-reduce of batch b+1 runs during batch b's scoring and batch b's count
    all-reduce + candidate all-gather during batch b+1's.  Results are identical to the sequential
    calls.  ``targets`` is a list of per-batch target tensors."""
    world = _world(group)
    if not world or len(hs) <= 1:
        return [sharded_rank_topk(h, table_shard, row_offset, t, k, group, mask_row0, scorer, counter, topk_fn)
                for h, t in zip(hs, targets)]
    S = _RankStages(table_shard, row_offset, k, group, mask_row0, scorer, counter, topk_fn, hs[0])
    out, prev = [], None
    pend = S.targets_start(hs[0], targets[0])
    for b in range(len(hs)):
        cur = pend
        if b + 1 < len(hs):
            pend = S.targets_start(hs[b + 1], targets[b + 1])
        sc = S.score_start(hs[b], cur)
        if prev is not None:
            out.append(S.finish(prev))
        prev = sc
    out.append(S.finish(prev))
    return out


class ShardedRankPipeline:
    """Cross-step form of ``sharded_rank_topk`` for a stream of batches (the
    exchange overlapped with the NEXT batch's work, without cutting a batch into smaller scoring
    launches).  ``submit(h, targets)`` runs the batch's target-logit all-reduce and its local
    scoring, issues its count all-reduce + candidate all-gather asynchronously and returns the
    PREVIOUS batch's result (None for the first), whose merge it enqueues after this batch's
    scoring; ``flush()`` returns the last batch's result.  Whatever the caller runs between two
    submits -- the next batch's transformer forward and hidden-state all-gather in bench.py's C5
    step -- runs under the collectives (RCCL's stream is FIFO: the next all-gather of h queues
    behind them, the compute stream does not).  Results are ``sharded_rank_topk``'s, bitwise.
    Without a process group there is nothing to overlap: ``submit`` returns the batch's own result
    once it is flushed, like any other rank."""

    def __init__(self, table_shard, row_offset, k=10, group=None, mask_row0=True,
                 scorer=None, counter=None, topk_fn=None):
        self.args = (table_shard, row_offset, k, group, mask_row0, scorer, counter, topk_fn)
        self.stages, self.prev = None, None

    @torch.no_grad()
    def submit(self, h, targets):
        table_shard, row_offset, k, group, mask_row0, scorer, counter, topk_fn = self.args
        if not _world(group):   # no exchange: the result is final at once, held for one submit
            cur = sharded_rank_topk(h, table_shard, row_offset, targets, k, group, mask_row0,
                                    scorer, counter, topk_fn)
            out, self.prev = self.prev, ("done", cur)
            return None if out is None else out[1]
        if self.stages is None:
            self.stages = _RankStages(table_shard, row_offset, k, group, mask_row0, scorer, counter, topk_fn, h)
        S = self.stages
        sc = S.score_start(h, S.targets_start(h, targets))
        out = self.flush()
        self.prev = ("pending", sc)
        return out

    @torch.no_grad()
    def flush(self):
        prev, self.prev = self.prev, None
        if prev is None:
            return None
        return prev[1] if prev[0] == "done" else self.stages.finish(prev[1])


def hr_ndcg(ranks, top_k=10):
    """HR@k / NDCG@k of SASRec/evaluate.py:36-47 (per-user float64 terms, then the mean)."""
    import numpy as np
    r = np.asarray(ranks.cpu() if torch.is_tensor(ranks) else ranks, dtype=np.int64)
    hit = r <= top_k
    ndcg = np.where(hit, 1.0 / np.log2(r.astype(np.float64) + 1.0), 0.0)
    return float(np.mean(hit.astype(np.float64))), float(np.mean(ndcg))
