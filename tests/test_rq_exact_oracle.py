"""Pin oracle/rq_exact.c (the exact-order restatement of RQVAE.get_indices) on the CPU.

The restatement spells out every fp32 rounding of the reference's CPU run (MKL's nn.Linear k
blocking, ATen's vectorised row sums, vq.py:71-75's association order), so it gives the same bits on
any host.  Pinned here against
  * every RQ golden fixture the reference itself produced (tests/golden/make_golden*.py imported
    /root/reference): encoder output z and the semantic IDs, bit for bit, BatchNorm included;
  * torch's own CPU ops in this (the fixture-generating) container on random shapes: nn.Linear at
    the reference's widths, the row sums, the vq.py distance argmin.
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import rq_exact, rq_oracle

RQ = ["rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256", "rq_calib_3x256",
      "rq_calib_wide_3x256"]


def _state(name):
    x, sd, out, meta = gl.rq_inputs(name)
    lin = sorted({int(k.split(".")[2]) for k in sd if k.startswith("encoder.mlp_layers") and k.endswith("weight")
                  and sd[k].ndim == 2})
    ws = [sd[f"encoder.mlp_layers.{i}.weight"] for i in lin]
    bs = [sd[f"encoder.mlp_layers.{i}.bias"] for i in lin]
    cbs = [sd[f"rq.vq_layers.{l}.embedding.weight"] for l in range(meta["L"])]
    return x, ws, bs, cbs, out, meta, sd


@pytest.mark.parametrize("name", RQ)
def test_exact_oracle_matches_reference_fixtures(name):
    x, ws, bs, cbs, out, meta, _ = _state(name)
    idx, z, best, gap = rq_exact.encode(x, ws, bs, cbs, with_detail=True)
    assert np.array_equal(idx, out["idx_full"]), f"{(idx != out['idx_full']).any(1).sum()} rows differ"
    if "z" in out:
        assert np.array_equal(z, out["z"])
    # the quantizer alone on the same latents, and the reference's own batch-64 call pattern
    assert np.array_equal(rq_exact.quantize(z, cbs), idx)
    if "idx_b64" in out:
        assert np.array_equal(out["idx_b64"], out["idx_full"])


def test_exact_oracle_batchnorm_fixture():
    x, sd, out, meta = gl.rq_inputs("rq_bn_3x256")
    ws = [sd[f"encoder.mlp_layers.{i}.weight"] for i in (1, 5, 9)]
    bs = [sd[f"encoder.mlp_layers.{i}.bias"] for i in (1, 5, 9)]
    bn = ([sd[f"encoder.mlp_layers.{i}.running_mean"] for i in (2, 6)],
          [sd[f"encoder.mlp_layers.{i}.running_var"] for i in (2, 6)],
          [sd[f"encoder.mlp_layers.{i}.weight"] for i in (2, 6)],
          [sd[f"encoder.mlp_layers.{i}.bias"] for i in (2, 6)], 1e-5)
    z = rq_exact.mlp(x, ws, bs, bn=bn)
    assert np.array_equal(z, out["z"])
    cbs = [sd[f"rq.vq_layers.{l}.embedding.weight"] for l in range(3)]
    assert np.array_equal(rq_exact.quantize(z, cbs), out["idx_full"])


def test_kblock_rule():
    assert rq_exact.kblock(768) == 384 and rq_exact.kblock(512) == 256 and rq_exact.kblock(383) == 383
    assert rq_exact.kblock(385) == 196 and rq_exact.kblock(700) == 352 and rq_exact.kblock(769) == 384
    assert rq_exact.kblock(384) == 384 and rq_exact.plan(64, 384, 64)[:2] == ("chain", 192)


def test_plan_rule_on_reference_widths():
    """MKL's order per call size for the reference encoder (main.py: 768 -> 256 -> 128 -> 32) and
    its quantizer (e = 32; K = 8 / 256 / 1024): one row = gemv16, 2-15 rows = small16 up to
    min(15, K / 24) rows, longer calls = the k-block chain -- all in the pinned envelope."""
    expect = {(768, 256): 15, (256, 128): 10, (128, 32): 5}
    for (k, n), top in expect.items():
        for m in range(1, 40):
            kind, kb, pinned = rq_exact.plan(m, k, n)
            assert pinned
            assert kind == ("gemv16" if m == 1 else "small16" if m <= top else "chain"), (m, k, n, kind)
            assert kb == (384 if k == 768 else k)
    for K in (8, 256, 1024):
        assert rq_exact.plan(1, 32, K)[0] == "gemv16" and rq_exact.plan(2, 32, K)[0] == "chain"
    assert rq_exact.plan(2, 64, 256)[0] == "small16" and rq_exact.plan(3, 64, 256)[0] == "chain"


# (rows, in, out): the reference's encoder widths (main.py: 768 -> 256 -> 128 -> 32, rqvae.py's
# default e_dim 64 / [512, 256, 128]) and odd widths across both sides of the 384 block edge.
LINEAR_SHAPES = [(64, 768, 256), (1000, 768, 256), (300, 256, 128), (100, 128, 32), (64, 512, 256),
                 (64, 400, 64), (64, 100, 300), (17, 768, 256), (16, 768, 256), (64, 128, 64)]


@pytest.mark.parametrize("m,k,n", LINEAR_SHAPES)
def test_exact_linear_matches_torch_cpu(m, k, n):
    rng = np.random.default_rng(m + k + n)
    x = rng.standard_normal((m, k), dtype=np.float32)
    w = rng.standard_normal((n, k), dtype=np.float32)
    b = rng.standard_normal(n, dtype=np.float32)
    ref = torch.nn.functional.linear(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b)).numpy()
    assert np.array_equal(rq_exact.linear(x, w, b), ref)
    ref0 = torch.nn.functional.linear(torch.from_numpy(x), torch.from_numpy(w)).numpy()
    assert np.array_equal(rq_exact.linear(x, w, None), ref0)
    refl = torch.nn.functional.leaky_relu(torch.from_numpy(ref)).numpy()
    assert np.array_equal(rq_exact.linear(x, w, b, act="leakyrelu"), refl)


@pytest.mark.parametrize("k,n", [(768, 256), (256, 128), (128, 32), (1000, 256), (1024, 256), (100, 64),
                                 (48, 8), (96, 96), (128, 128)])
def test_exact_linear_small_calls_match_torch_cpu(k, n):
    """Calls of 1..17 rows: MKL's one-row gemv order, its 2-15-row small-kernel order and the chain
    past the switch point, against torch's own CPU F.linear here (8 threads, the fixture host)."""
    torch.set_num_threads(8)
    rng = np.random.default_rng(k * 3 + n)
    w = rng.standard_normal((n, k), dtype=np.float32) * 0.05
    b = rng.standard_normal(n, dtype=np.float32) * 0.1
    for m in range(1, 18):
        x = rng.standard_normal((m, k), dtype=np.float32)
        ref = torch.nn.functional.linear(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b)).numpy()
        got = rq_exact.linear(x, w, b)
        if rq_exact.plan(m, k, n)[2]:
            assert np.array_equal(got, ref), (m, k, n, rq_exact.plan(m, k, n))


def test_pinned_envelope_random_shapes():
    """Random (M, K, N) inside rqx_plan_pinned's envelope: the restated order is torch's bit for
    bit (scripts/mkl_order_probe.py runs the long version of this sweep)."""
    torch.set_num_threads(8)
    rng = np.random.default_rng(7)
    checked = 0
    while checked < 60:
        m = int(rng.choice([1, rng.integers(2, 16), rng.integers(16, 300)]))
        k = int(rng.choice([rng.integers(1, 384), 128 * rng.integers(1, 7), rng.integers(24, 1100)]))
        n = int(rng.choice([rng.integers(2, 300), 32 * rng.integers(1, 9)]))
        if not rq_exact.plan(m, k, n)[2] or m * n * k > 2e7:
            continue
        x = rng.standard_normal((m, k), dtype=np.float32)
        w = rng.standard_normal((n, k), dtype=np.float32) * 0.05
        b = rng.standard_normal(n, dtype=np.float32) * 0.1
        ref = torch.nn.functional.linear(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b)).numpy()
        assert np.array_equal(rq_exact.linear(x, w, b), ref), (m, k, n, rq_exact.plan(m, k, n))
        checked += 1


@pytest.mark.parametrize("n", [1, 2, 3, 5, 15, 16])
@pytest.mark.parametrize("e,Ks", [(32, [256, 256, 256]), (32, [8, 8, 8]), (64, [256, 64]), (96, [256]),
                                  (128, [256, 512])])
def test_exact_quantize_small_calls_match_torch_cpu(n, e, Ks):
    """The quantizer's matmul (vq.py:73) at call sizes where MKL leaves the chain order (one row;
    e >= 48 also 2 rows), against the vq.py formula run by torch on the same call."""
    torch.set_num_threads(8)
    rng = np.random.default_rng(n * 31 + e)
    z = rng.standard_normal((n, e), dtype=np.float32)
    cbs = [(z[rng.integers(0, n, K)] + 0.3 * rng.standard_normal((K, e), dtype=np.float32)).astype(np.float32)
           for K in Ks]
    ref_idx, _, _ = rq_oracle.rq_quantize(torch.from_numpy(z), [torch.from_numpy(c) for c in cbs],
                                           return_detail=True)
    idx, best, gap = rq_exact.quantize(z, cbs, with_detail=True)
    assert np.array_equal(idx, ref_idx.numpy())
    # the distances themselves, not only the argmin: level 0's d row of vq.py:71-73
    d = rq_oracle.vq_level(torch.from_numpy(z), torch.from_numpy(cbs[0]))[2]
    assert np.array_equal(best[:, 0], d.min(1).values.numpy())


SMALL = ["rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256"]


@pytest.mark.parametrize("name", SMALL)
def test_exact_oracle_matches_reference_small_calls(name):
    """The reference's own get_indices at call sizes 1..17 (make_golden_smallbatch.py) and its
    batch-64 loop over a 707-item catalog (a 3-row tail): IDs and, for 3x256, the encoder output
    bit for bit per call."""
    x, ws, bs, cbs, _, meta, _ = _state(name)
    sm = np.load(f"{gl.HERE}/{name}_small.npz", allow_pickle=False)
    for m in range(1, 18):
        idx, starts = sm[f"small_M{m}"], sm[f"small_starts_M{m}"]
        for wi, s in enumerate(starts[:48]):
            o_idx, o_z, _, _ = rq_exact.encode(x[s:s + m], ws, bs, cbs, with_detail=True)
            assert np.array_equal(o_idx, idx[wi]), (m, s)
            if f"z_M{m}" in sm.files:
                assert np.array_equal(o_z, sm[f"z_M{m}"][wi]), (m, s)
    c = np.load(f"{gl.HERE}/csv_bert.npz", allow_pickle=False)
    cat, sha = gl.synth_items(707, c["mu"], c["sigma"], 11)
    assert np.array_equal(rq_exact.encode_batches(cat, ws, bs, cbs, 64), sm["b64_707"])
    assert np.array_equal(rq_exact.encode(cat, ws, bs, cbs), sm["b64_707_full"])


def test_small_call_bits_differ_from_long_call():
    """The small-call orders are not a no-op: the reference's encoder output of a 1..15-row call
    differs from the same rows inside a long call (so the fixtures above discriminate)."""
    x, ws, bs, cbs, out, meta, _ = _state("rq_syn_3x256")
    sm = np.load(f"{gl.HERE}/rq_syn_3x256_small.npz", allow_pickle=False)
    z_long = out["z"]
    for m in (1, 2, 7, 15):
        starts = sm[f"small_starts_M{m}"]
        zs = sm[f"z_M{m}"]
        moved = sum(int((zs[wi] != z_long[s:s + m]).any()) for wi, s in enumerate(starts))
        assert moved > len(starts) // 2, (m, moved)
    zs = sm["z_M16"]
    assert all(np.array_equal(zs[wi], z_long[s:s + 16]) for wi, s in enumerate(sm["small_starts_M16"]))


@pytest.mark.parametrize("e", [1, 7, 8, 16, 20, 24, 32, 40, 48, 64, 96, 128])
def test_exact_rowsq_matches_torch_cpu(e):
    rng = np.random.default_rng(e)
    x = rng.standard_normal((5000, e), dtype=np.float32) * rng.uniform(0.1, 3, (5000, 1)).astype(np.float32)
    ref = torch.sum(torch.from_numpy(x) ** 2, dim=1).numpy()
    assert np.array_equal(rq_exact.rowsq(x), ref)


@pytest.mark.parametrize("e,Ks", [(32, [256, 256, 256]), (16, [300, 7]), (20, [64, 33]), (64, [1024, 1, 5]),
                                  (32, [8, 8, 8])])
def test_exact_quantize_matches_torch_cpu(e, Ks):
    """The quantizer alone against the vq.py formula run by torch (oracle/rq_oracle.py), including
    the reference's own near-tie-heavy uniform(+-1/K) codebooks."""
    rng = np.random.default_rng(e * 7 + len(Ks))
    z = rng.standard_normal((4096, e), dtype=np.float32)
    cbs = [rng.uniform(-1.0 / K, 1.0 / K, (K, e)).astype(np.float32) for K in Ks]
    ref = rq_oracle.rq_quantize(torch.from_numpy(z), [torch.from_numpy(c) for c in cbs]).numpy()
    assert np.array_equal(rq_exact.quantize(z, cbs), ref)


def test_exact_mlp_batchnorm_and_activations_match_torch_cpu():
    """MLPLayers eval with BatchNorm1d (running statistics, affine) and LeakyReLU / none."""
    torch.manual_seed(3)
    dims = [96, 64, 48, 16]
    lins = [torch.nn.Linear(a, b) for a, b in zip(dims[:-1], dims[1:])]
    bns = [torch.nn.BatchNorm1d(d) for d in dims[1:-1]]
    with torch.no_grad():
        for bn in bns:
            bn.running_mean.normal_(0, 0.3)
            bn.running_var.uniform_(0.5, 2.0)
            bn.weight.normal_(1, 0.1)
            bn.bias.normal_(0, 0.1)
            bn.eval()
    x = torch.randn(700, dims[0])
    for act, fn in (("relu", torch.relu), ("leakyrelu", torch.nn.functional.leaky_relu), ("none", lambda t: t)):
        with torch.no_grad():
            h = x
            for i, lin in enumerate(lins):
                h = lin(h)
                if i < len(bns):
                    h = fn(bns[i](h))
        bn = ([b.running_mean.numpy() for b in bns], [b.running_var.numpy() for b in bns],
              [b.weight.detach().numpy() for b in bns], [b.bias.detach().numpy() for b in bns], 1e-5)
        z = rq_exact.mlp(x.numpy(), [l.weight.detach().numpy() for l in lins], [l.bias.detach().numpy() for l in lins],
                         bn=bn, act=act)
        assert np.array_equal(z, h.numpy()), act
