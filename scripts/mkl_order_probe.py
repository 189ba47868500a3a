"""Characterise / re-check MKL's sgemm accumulation order on THIS host (container-only tool).

The reference's encoder runs torch's CPU nn.Linear (RQ-VAE/models/layers.py:23 -> addmm -> MKL
sgemm) and its quantizer torch.matmul (vq.py:73).  oracle/rq_exact.c restates their order as a
function of the call's (M rows, K inner, N outputs) -- rqx_plan -- and claims an envelope where that
restatement is verified (rqx_plan_pinned).  This script draws random shapes, runs torch's CPU op and
the restatement, and reports disagreements split by pinned / unpinned:

    python scripts/mkl_order_probe.py --samples 2000 --seed 1

How the orders were found (kept for the record): FPRev-style probes -- x = 1, w = +B / -B at two
positions and 1 elsewhere (B = 2^40, so a +-B pair cancels only after both have absorbed every 1
added to their partial sums) give the size of the smallest subtree holding both positions; the
matrix of those sizes is the summation tree (printed by --tree M K N).
"""
import argparse
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import rq_exact  # noqa: E402

BIG = 2.0 ** 40


def lca_sizes(M, K, N, row=0):
    """S[a, b] = leaves in the smallest subtree holding products a and b (leaf K = the bias)."""
    L = K + 1
    pairs = [(a, b) for a in range(L) for b in range(a + 1, L)]
    S = np.zeros((L, L), np.int64)
    for s in range(0, len(pairs), N):
        ch = pairs[s:s + N]
        W = torch.ones(N, K)
        bias = torch.ones(N)
        for j, (a, b) in enumerate(ch):
            for leaf, v in ((a, BIG), (b, -BIG)):
                if leaf == K:
                    bias[j] = v
                else:
                    W[j, leaf] = v
        y = torch.nn.functional.linear(torch.ones(M, K), W, bias)
        for j, (a, b) in enumerate(ch):
            S[a, b] = S[b, a] = L - int(y[row, j].item())
    return S


def tree(S, leaves):
    if len(leaves) == 1:
        return leaves[0]
    n = len(leaves)
    comp, seen = [], set()
    for a in leaves:
        if a in seen:
            continue
        stack, c = [a], []
        seen.add(a)
        while stack:
            u = stack.pop()
            c.append(u)
            for v in leaves:
                if v not in seen and S[u, v] < n:
                    seen.add(v)
                    stack.append(v)
        comp.append(sorted(c))
    if len(comp) == 1:
        return ("?",)
    return tuple(tree(S, c) for c in comp)


def check(M, K, N, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) * 0.05
    b = torch.randn(N, generator=g) * 0.1
    ref = torch.nn.functional.linear(x, w, b).numpy()
    return bool(np.array_equal(rq_exact.linear(x.numpy(), w.numpy(), b.numpy()), ref))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=500)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max-work", type=float, default=1e8, help="max M*N*K per sample")
    ap.add_argument("--tree", type=int, nargs=3, metavar=("M", "K", "N"))
    a = ap.parse_args()
    torch.set_num_threads(8)
    if a.tree:
        M, K, N = a.tree
        print(tree(lca_sizes(M, K, N), list(range(K + 1))))
        return
    rng = random.Random(a.seed)
    stats = {}
    bad = []
    for t in range(a.samples):
        M = rng.choice([1, rng.randint(2, 15), rng.randint(16, 300), rng.randint(256, 2048)])
        K = rng.choice([rng.randint(1, 400), rng.randint(1, 1100), 128 * rng.randint(1, 32)])
        N = rng.choice([rng.randint(2, 600), 8 * rng.randint(1, 128), 2 ** rng.randint(3, 10)])
        if M * N * K > a.max_work:
            continue
        kind, kb, pinned = rq_exact.plan(M, K, N)
        ok = check(M, K, N, t)
        key = (kind, pinned)
        s = stats.setdefault(key, [0, 0])
        s[0] += 1
        s[1] += ok
        if pinned and not ok:
            bad.append((M, K, N, kind, kb))
    for (kind, pinned), (n, ok) in sorted(stats.items()):
        print(f"{kind:8s} pinned={pinned!s:5s} samples={n:5d} match={ok:5d}")
    print("pinned mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
