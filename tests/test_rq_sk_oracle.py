"""use_sk=True / code-emission oracle pinned against the reference's golden fixtures (CPU), and the
product's host-side collision grouping / dedup against the oracle."""
import numpy as np
import torch

import golden_lib as gl
from oracle import rq_oracle


def _case(name):
    sd, out, meta = gl.load(name)
    if name == "rq_sk_csv_3x8":
        x, _, _, _ = gl.rq_inputs("rq_csv_3x8")
    else:
        c = np.load(gl.os.path.join(gl.HERE, "csv_bert.npz"), allow_pickle=False)
        x, sha = gl.synth_items(meta["n"], c["mu"], c["sigma"], meta["x_seed"])
        assert sha == meta["x_sha256"]
    ws, bs, cbs = rq_oracle.state_to_lists({k: torch.from_numpy(v) for k, v in sd.items()}, meta["L"])
    return torch.from_numpy(x), ws, bs, cbs, out, meta


def test_oracle_infer_codes_matches_reference_csv():
    x, ws, bs, cbs, out, meta = _case("rq_sk_csv_3x8")
    codes, final, rounds = rq_oracle.infer_codes(x, ws, bs, cbs, [0.01] * meta["L"], meta["sk_iters"])
    assert np.array_equal(final, out["final"]) and len(rounds) == meta["rounds"]
    assert len(np.unique(final, axis=0)) == len(final)


def test_oracle_sinkhorn_all_levels_matches_reference():
    for name in ("rq_sk_csv_3x8", "rq_sk_syn_3x16"):
        x, ws, bs, cbs, out, meta = _case(name)
        ptr, rows = out["all_ptr"], out["all_rows"]
        for g in range(len(ptr) - 1)[:40]:
            r = rows[ptr[g]:ptr[g + 1]]
            got = rq_oracle.get_indices_sk(x[r], ws, bs, cbs, [0.01] * meta["L"], meta["sk_iters"])
            assert np.array_equal(got.numpy(), out["all_out"][ptr[g]:ptr[g + 1]])


def test_product_grouping_and_dedup_equal_oracle():
    from gr_amd.infer import collision_groups, dedup_codes
    rng = np.random.default_rng(0)
    for _ in range(20):
        codes = rng.integers(0, 3, size=(50, 3))
        assert collision_groups(codes) == rq_oracle.collision_groups(codes)
        assert np.array_equal(dedup_codes(codes), rq_oracle.dedup_codes(codes))
    _, out, _ = gl.load("rq_sk_syn_3x16")
    assert np.array_equal(dedup_codes(out["codes"]), out["final"])
