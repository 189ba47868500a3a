"""CPU restatement of the SASRec evaluation tail (test infrastructure only).

SASRec/evaluate.py:26-47: padding column masked to -1e9, strict rank
``#{j : logit_j > logit_target} + 1`` taken from the same logits tensor, HR@k / NDCG@k
accumulated per user in Python and averaged with ``np.mean``.
"""
import numpy as np
import torch


def ranks_from_logits(logits, targets):
    """evaluate.py:27-32 on a copy of ``logits`` (the caller's tensor is not mutated)."""
    lg = logits.clone()
    lg[:, 0] = -1e9
    t = lg.gather(1, targets.view(-1, 1))
    return (lg > t).sum(dim=1) + 1


def hr_ndcg(ranks, top_k=10):
    """evaluate.py:36-47: per-user Python accumulation then ``np.mean``."""
    ht, ndcg = [], []
    for r in np.asarray(ranks):
        if r <= top_k:
            ht.append(1)
            ndcg.append(1 / np.log2(r + 1))
        else:
            ht.append(0)
            ndcg.append(0)
    return float(np.mean(ht)), float(np.mean(ndcg))
