"""SASRec evaluation harness on the gfx950 kernels — SASRec/evaluate.py:10-89 and the multi-k
evaluation of SASRec/train.py:33-56.

The reference computes ``logits = model.predict(x)`` ([B, N+1] fp32), masks column 0 with -1e9,
gathers the target's logit and counts strictly greater logits (evaluate.py:26-32).  Here the rank
of a batch is ONE C-ABI call, ``ops.sasrec_rank`` (``gr_sasrec_rank_f32``): the last hidden state
from the fused SASRec forward, then the target logit and the strict-'>' count straight from the
scoring kernel's MFMA tiles — the [B, N+1] logits are never written (``materialize=True`` runs
the reference's predict + rank sequence instead; both give the same ranks,
tests/test_evaluate_gpu.py).  HR@k / NDCG@k are then formed on the host in float64 with the
reference's values (its per-user lists built as arrays, the same ``np.mean``, evaluate.py:35-47;
bitwise the loop, tests/test_data.py).
"""
import csv
import os

import numpy as np
import torch

from . import ops
from .data import SASRecDataset


def rank_batch(model, input_ids, targets, materialize=False):
    """Strict 1-based rank of each target over the full catalog with column 0 masked
    (SASRec/evaluate.py:26-32) for one batch on the model's device."""
    if materialize:
        logits = model.predict(input_ids)
        logits[:, 0] = -1e9
        t = logits.gather(1, targets.unsqueeze(1))
        return (logits > t).sum(dim=1) + 1
    if model.d not in (16, 32, 64, 128):   # the fused kernels' widths; others: predict + rank kernel
        return ops.rank(model.predict(input_ids), targets, mask_col0=True)
    # forward + target logit + strict count in one C-ABI call (gr_sasrec_rank_f32)
    return ops.sasrec_rank(model._binding(input_ids), input_ids, targets, mask_col0=True)


def _ndcg_terms(ranks, top_k):
    """The per-user lists of evaluate.py:36-42 as float64 arrays, element for element: a hit is 1,
    its NDCG term ``1 / np.log2(r + 1)`` evaluated exactly as the reference's loop evaluates it (numpy
    int64 scalar r, scalar log2, true divide) -- once per distinct rank <= top_k, then gathered --
    and every miss 0.  np.mean of these arrays is np.mean of the reference's lists (the lists are
    converted to the same float64 arrays), without the per-user Python loop (~10 ms at 95,423 users)."""
    r = np.asarray(ranks).astype(np.int64, copy=False).reshape(-1)
    hit = r <= top_k
    lut = np.zeros(max(int(top_k), 0) + 2, dtype=np.float64)
    for v in np.unique(r[hit]):
        lut[int(v)] = 1 / np.log2(np.int64(v) + 1)
    ndcg = np.where(hit, lut[np.clip(r, 0, len(lut) - 1)], 0.0)
    return hit.astype(np.float64), ndcg


def hr_ndcg(ranks, top_k):
    """evaluate.py:35-47: per-user hit / 1/log2(r+1), averaged with np.mean (float64)."""
    ht, ndcg = _ndcg_terms(ranks, top_k)
    if ht.size == 0:
        return float(np.mean([])), float(np.mean([]))
    return float(np.mean(ht)), float(np.mean(ndcg))


def multi_k(ranks, topk_list, targets=None):
    """SASRec/train.py:33-56: {k: HR@k}, {k: NDCG@k} for every k of ``topk_list``.  With ``targets``
    the users whose target is 0 are dropped first (train.py:42-45 ``valid_mask``)."""
    ranks = np.asarray(ranks)
    if targets is not None:
        ranks = ranks[np.asarray(targets) != 0]
    hk, nk = {}, {}
    for k in topk_list:   # the per-user lists of train.py:46-50 as arrays (_ndcg_terms), same np.mean
        ht, nd = _ndcg_terms(ranks, k)
        hk[k] = float(np.mean(ht)) if ht.size else 0.0
        nk[k] = float(np.mean(nd)) if nd.size else 0.0
    return hk, nk


@torch.no_grad()
def evaluate(params, dataset=None, model=None, materialize=False, save_csv=True, with_multi_k=False):
    """SASRec/evaluate.py:evaluate(params).  ``dataset`` / ``model`` may be passed in directly (the
    reference builds them from ``params['data_path']`` / ``params['ckpt']``); checkpoints are read
    with ``torch.load(weights_only=True)``.  Returns ``(results, ranks)``: ``results`` is exactly the
    reference's dict {"Hit@top_k", "NDCG@top_k"} (evaluate.py:51), which is also all the CSV row
    carries (evaluate.py:52, 57-89).  ``with_multi_k``: a third value, {"Hit@k", "NDCG@k"} for every
    k of ``params['topk_list']`` with train.py:33-56's semantics (target-0 users dropped) -- kept
    out of ``results`` and out of the CSV so both keep the reference's schema."""
    from .sasrec import SASRec
    device = torch.device(params["device"])
    if dataset is None:
        dataset = SASRecDataset(params["data_path"], max_len=params["max_len"], mode="test", params=params)
    if model is None:
        model = SASRec(dataset.item_num, params).to(device)
        model.load_state_dict(torch.load(params["ckpt"], map_location=device, weights_only=True))
    model.eval()
    ranks, tgts = [], []
    for input_ids, target in dataset.batches(params.get("eval_batch_size", 128)):
        ranks.append(rank_batch(model, input_ids.to(device), target.to(device), materialize))
        tgts.append(target)
    if device.type == "cuda":
        ops.check_errors(device)     # out-of-range ids flagged by the kernels (IndexError)
    ranks = torch.cat(ranks).cpu().numpy() if ranks else np.zeros(0, np.int64)
    tgts = torch.cat(tgts).numpy() if tgts else np.zeros(0, np.int64)
    top_k = params.get("top_k", 10)
    hit, ndcg = hr_ndcg(ranks, top_k)
    results = {f"Hit@{top_k}": hit, f"NDCG@{top_k}": ndcg}
    if save_csv and params.get("params_path"):
        save_results_to_csv(params, results)
    if not with_multi_k:
        return results, ranks
    multi = {}
    if params.get("topk_list"):        # train.py:33-56 semantics: target-0 users dropped
        hk, nk = multi_k(ranks, params["topk_list"], tgts)
        for k in params["topk_list"]:
            multi[f"Hit@{k}"] = hk[k]
            multi[f"NDCG@{k}"] = nk[k]
    return results, ranks, multi


@torch.no_grad()
def train_evaluate(model, test_loader, params, device):
    """SASRec/train.py:33-56 ``evaluate(model, test_loader, params, device)``: users with target 0
    dropped (``valid_mask``, :42-45), strict ranks from the fused kernels, HR@k / NDCG@k for every
    k of ``params['topk_list']``.  Leaves the model in train mode like the reference (:53)."""
    model.eval()
    ranks = []
    for input_ids, target_item in test_loader:
        input_ids = input_ids.to(device)
        target_item = target_item.to(device)
        valid = target_item != 0
        if not bool(valid.any()):
            continue
        ranks.append(rank_batch(model, input_ids[valid], target_item[valid]))
    ops.check_errors(torch.device(device))
    model.train()
    r = torch.cat(ranks).cpu().numpy() if ranks else np.zeros(0, np.int64)
    return multi_k(r, params["topk_list"])


def save_results_to_csv(params, results):
    """evaluate.py:57-89: append task_id, the hyper-parameters and the metrics (6 decimals)."""
    csv_path = params["params_path"]
    os.makedirs(os.path.dirname(csv_path) if os.path.dirname(csv_path) else ".", exist_ok=True)
    data = {"task_id": params.get("task_id")}
    for name in ["d", "num_blocks", "num_heads", "dropout", "lr", "batch_size", "epochs",
                 "mlp_layer", "max_len", "top_k"]:
        if name in params:
            data[name] = params[name]
    for key, value in results.items():
        data[key] = f"{value:.6f}"
    exists = os.path.exists(csv_path)
    with open(csv_path, "a", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        if not exists:
            w.writerow(data.keys())
        w.writerow(data.values())
