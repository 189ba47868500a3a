"""RQVAE.get_indices(use_sk=True) (Sinkhorn collision re-encode) and the infer.py code emission on
the GPU vs the reference's golden fixtures (tests/golden/make_golden_sk.py).

Bar: semantic IDs equal to the reference's, every row.  The Sinkhorn runs in float64 like the
reference; its inputs are the fp32 distances, so a row could in principle move where the reference
itself sits on a near-tie, but none does on these fixtures (40,447 re-encoded rows in 10,493
groups: 0 differ, profiles/r02_parity_counts.json), and the tests hold that exactly."""
import numpy as np
import pytest
import torch

import golden_lib as gl
from test_rq_sk_oracle import _case

pytestmark = pytest.mark.gpu
CASES = ["rq_sk_csv_3x8", "rq_sk_syn_3x16"]


def model_of(name, dev, eps):
    from gr_amd import RQVAE
    sd, out, meta = gl.load(name)
    m = RQVAE(in_dim=768, num_emb_list=[meta["K"]] * meta["L"], e_dim=32, layers=[256, 128],
              dropout_prob=0.1, sk_epsilons=list(eps), sk_iters=meta["sk_iters"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    return m.to(dev).eval()


@pytest.mark.parametrize("name", CASES)
def test_grouped_sinkhorn_reencode_matches_reference(name, dev, parity_log):
    """Every collision round's groups, all in one launch, against the reference's per-group calls."""
    x, _, _, _, out, meta = _case(name)
    L = meta["L"]
    m = model_of(name, dev, [0.0] * (L - 1) + [0.01])       # infer.py:109-110
    rows, ptr = out["round_rows"], out["round_ptr"]
    sizes = np.diff(ptr)
    got = m.get_indices_groups(x[torch.from_numpy(rows)].to(dev), sizes.tolist()).cpu().numpy()
    bad = (got != out["round_out"]).any(1)
    parity_log(kind="rq_sinkhorn_reencode", fixture=name, levels="last level Sinkhorn (infer.py:109-110)",
               rows=len(bad), groups=len(sizes), rows_differ=int(bad.sum()), cap=0)
    assert bad.sum() == 0
    # a single group through the drop-in get_indices(use_sk=True) = the same rows of the launch
    r0 = torch.from_numpy(rows[ptr[0]:ptr[1]])
    assert np.array_equal(m.get_indices(x[r0].to(dev), use_sk=True).cpu().numpy(), got[:ptr[1]])


@pytest.mark.parametrize("name", CASES)
def test_sinkhorn_every_level_matches_reference(name, dev, parity_log):
    x, _, _, _, out, meta = _case(name)
    m = model_of(name, dev, [0.01] * meta["L"])
    rows, ptr = out["all_rows"], out["all_ptr"]
    got = m.get_indices_groups(x[torch.from_numpy(rows)].to(dev), np.diff(ptr).tolist()).cpu().numpy()
    bad = (got != out["all_out"]).any(1)
    parity_log(kind="rq_sinkhorn_reencode", fixture=name, levels="every level Sinkhorn", rows=len(bad),
               groups=len(ptr) - 1, rows_differ=int(bad.sum()), cap=0)
    assert bad.sum() == 0


def test_infer_code_emission_matches_reference(dev, tmp_path, parity_log):
    """RQ-VAE/infer.py end to end on the config-1 items: codes, 30 collision rounds, dedup digit,
    .npy + mapping json."""
    import json
    from gr_amd.infer import generate_codes, save_codes
    x, _, _, _, out, meta = _case("rq_sk_csv_3x8")
    m = model_of("rq_sk_csv_3x8", dev, [0.01] * meta["L"])
    codes, final, stats = generate_codes(m, x, dev)
    parity_log(kind="rq_code_emission", fixture="rq_sk_csv_3x8", rows=len(final),
               rows_differ_codes=int((codes != out["codes"]).any(1).sum()),
               rows_differ_final=int((final != out["final"]).any(1).sum()),
               rounds=stats["rounds"], ref_rounds=meta["rounds"])
    assert np.array_equal(codes, out["codes"]) and np.array_equal(final, out["final"])
    assert stats["rounds"] == meta["rounds"]
    f = str(tmp_path / "codes.npy")
    mp = save_codes(final, f)
    assert np.array_equal(np.load(f), final)
    assert json.load(open(mp))["3"] == final[3].tolist()


@pytest.mark.parametrize("B,K", [(64, 8), (64, 256), (2048, 8), (1500, 64)])
def test_sinkhorn_batch_shapes_vs_oracle(B, K, dev, parity_log):
    """One group of B rows (a training batch) at every level, against the oracle's restatement of
    vq.py:63-99 / layers.py:85-108 level by level: the LDS-resident matrix (64 x 8, 64 x 256), the
    large-group LDS loop (2048 x 8) and the workspace-resident matrix (1500 x 64)."""
    from gr_amd import ops
    from oracle import rq_oracle
    g = torch.Generator().manual_seed(B + K)
    z = torch.randn(B, 32, generator=g)
    cbs = [torch.randn(K, 32, generator=g) * 0.8 for _ in range(3)]
    got = ops.rq_quantize_sk(z.to(dev), [c.to(dev) for c in cbs], [0.01, 0.0, 0.01], 50).cpu()
    r, ref = z.clone(), []
    for c, eps in zip(cbs, [0.01, 0.0, 0.01]):
        xq, ind = rq_oracle.vq_level_sk(r, c, eps, 50)
        ref.append(ind)
        r = r - xq
    ref = torch.stack(ref, -1)
    bad = int((got != ref).any(1).sum())
    parity_log(kind="rq_sinkhorn_batch", shape=f"B{B} K{K}", rows=B, rows_differ=bad, cap=0)
    assert bad == 0
