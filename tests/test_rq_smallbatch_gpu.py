"""RQ-VAE get_indices on the GPU at the reference's SMALL call sizes (1-15 rows).

MKL's CPU sgemm takes other accumulation orders for calls of 1-15 rows (oracle/rq_exact.c rqx_plan:
one row = 16-lane gemv, 2-15 rows = 16-lane small kernel), so the reference's encoder output and
IDs depend on the call's row count there.  The reference makes such calls for the tail of its
DataLoader(bs=64) loop (RQ-VAE/infer.py:84-95, generate_code.py:78-88) and for small collision
groups (infer.py:121-122).  Bar: bit-exact IDs and encoder output against the reference's own
small calls (tests/golden/*_small.npz, make_golden_smallbatch.py) and against the exact-order
oracle on near-tie codebooks where the small-call bits move most IDs.
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import rq_exact
from test_rq_gpu import build_model

pytestmark = pytest.mark.gpu
SMALL = ["rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256"]


def _lists(sd, L):
    ws = [sd[f"encoder.mlp_layers.{i}.weight"] for i in (1, 4, 7)]
    bs = [sd[f"encoder.mlp_layers.{i}.bias"] for i in (1, 4, 7)]
    return ws, bs, [sd[f"rq.vq_layers.{l}.embedding.weight"] for l in range(L)]


@pytest.mark.parametrize("name", SMALL)
def test_small_calls_match_reference(name, dev, parity_log):
    x, sd, _, meta = gl.rq_inputs(name)
    sm = np.load(f"{gl.HERE}/{name}_small.npz", allow_pickle=False)
    m = build_model(meta, sd, dev)
    from gr_amd import ops
    lin = m.encoder.linears()
    xg = torch.from_numpy(x).to(dev)
    rows = differ = zdiffer = 0
    for M in range(1, 18):
        idx_ref, starts = sm[f"small_M{M}"], sm[f"small_starts_M{M}"]
        zref = sm[f"z_M{M}"] if f"z_M{M}" in sm.files else None
        for wi, s in enumerate(starts[:48]):
            got = m.get_indices(xg[s:s + M]).cpu().numpy()
            differ += int((got != idx_ref[wi]).any(1).sum())
            rows += M
            if zref is not None:
                _, z = ops.rq_encode(xg[s:s + M], [l.weight for l in lin], [l.bias for l in lin], m.rq.codebooks(),
                                     with_z=True)
                zdiffer += int((z.cpu().numpy() != zref[wi]).any(1).sum())
    parity_log(kind="rq_small_calls", fixture=name, rows=rows, rows_differ=differ, z_rows_differ=zdiffer)
    assert differ == 0 and zdiffer == 0


@pytest.mark.parametrize("name", SMALL)
def test_batch64_loop_with_short_tail(name, dev, parity_log):
    """The reference's batch-64 loop over the 707-item catalog (11 full batches + a 3-row tail):
    get_indices_batched (two launches) and the per-batch loop both give the reference's IDs."""
    _, sd, _, meta = gl.rq_inputs(name)
    sm = np.load(f"{gl.HERE}/{name}_small.npz", allow_pickle=False)
    c = np.load(f"{gl.HERE}/csv_bert.npz", allow_pickle=False)
    cat, _ = gl.synth_items(707, c["mu"], c["sigma"], 11)
    m = build_model(meta, sd, dev)
    cg = torch.from_numpy(cat).to(dev)
    got = m.get_indices_batched(cg, 64).cpu().numpy()
    loop = torch.cat([m.get_indices(cg[i:i + 64]) for i in range(0, 707, 64)]).cpu().numpy()
    parity_log(kind="rq_b64_707", fixture=name, rows=707, rows_differ=int((got != sm["b64_707"]).any(1).sum()))
    assert np.array_equal(got, sm["b64_707"]) and np.array_equal(loop, sm["b64_707"])
    assert np.array_equal(m.get_indices(cg).cpu().numpy(), sm["b64_707_full"])


@pytest.mark.parametrize("fused", [1, 0])
def test_small_calls_on_knife_edge_codebooks(dev, fused, parity_log):
    """Codebooks scattered tightly around each row's LONG-call latent: the small-call bits change
    ~80 % of the IDs there (checked below), so only the small-call order reproduces the oracle."""
    from gr_amd import RQVAE, _lib
    x, sd, _, meta = gl.rq_inputs("rq_syn_3x256")
    ws, bs, _ = _lists(sd, 3)
    rng = np.random.default_rng(5)
    _lib.set_option("rq_fused", fused)
    try:
        rows = differ = moved = 0
        for M in (1, 2, 3, 5, 8, 11, 15, 16):
            for s in rng.integers(0, 8000, 6):
                zl = rq_exact.mlp(x[s:s + 64], ws, bs)[:M]
                cbs = [(np.repeat(zl, 256 // M + 1, 0)[:256] + 1e-4 * np.abs(zl).mean()
                        * rng.standard_normal((256, 32))).astype(np.float32) for _ in range(3)]
                ref = rq_exact.encode(x[s:s + M], ws, bs, cbs)
                moved += int((ref != rq_exact.quantize(zl, cbs, call_m=64)).any(1).sum())
                m = RQVAE(in_dim=768, num_emb_list=[256] * 3, e_dim=32, layers=[256, 128], sk_epsilons=[0.0] * 3)
                with torch.no_grad():
                    for lin, w, b in zip(m.encoder.linears(), ws, bs):
                        lin.weight.copy_(torch.from_numpy(w))
                        lin.bias.copy_(torch.from_numpy(b))
                    for q, cb in zip(m.rq.vq_layers, cbs):
                        q.embedding.weight.copy_(torch.from_numpy(cb))
                m = m.to(dev).eval()
                got = m.get_indices(torch.from_numpy(x[s:s + M]).to(dev)).cpu().numpy()
                differ += int((got != ref).any(1).sum())
                rows += M
        parity_log(kind="rq_knife_edge", path="fused" if fused else "layerwise", rows=rows, rows_differ=differ,
                   rows_moved_by_small_call_order=moved)
        assert moved > rows // 4, "the codebooks do not discriminate the call orders"
        assert differ == 0
    finally:
        _lib.set_option("rq_fused", 1)


def test_collision_groups_use_each_groups_call_order(dev, parity_log):
    """get_indices_groups: every group is one reference call (its own MKL order), as the per-group
    loop of RQ-VAE/infer.py:116-127; the encoder half against rq_exact per group (the chain-order
    groups batched into one MFMA-kernel call, the small-call groups on the per-row kernel)."""
    x, sd, _, meta = gl.rq_inputs("rq_syn_3x256")
    ws, bs, cbs = _lists(sd, 3)
    m = build_model(meta, sd, dev)
    rng = np.random.default_rng(3)
    # 1-19-row groups (their own small-call orders, the per-row kernel) mixed with groups of >= 16 rows
    # that share one k-block-chain order (one MFMA-kernel call over all of them)
    sizes = [int(v) for v in rng.integers(1, 20, 40)] + [16, 64, 33, 100]
    sizes = [sizes[i] for i in rng.permutation(len(sizes))]
    rows = rng.permutation(len(x))[:sum(sizes)]
    z = m.encoder(torch.from_numpy(x[rows]).to(dev), group_sizes=sizes).cpu().numpy()
    ref, off = [], 0
    for g in sizes:
        ref.append(rq_exact.mlp(x[rows[off:off + g]], ws, bs))
        off += g
    ref = np.concatenate(ref)
    parity_log(kind="rq_group_encoder", rows=len(rows), rows_differ=int((z != ref).any(1).sum()))
    assert np.array_equal(z, ref)
    # the use_sk=True re-encode of those groups against the per-group reference loop
    from gr_amd import RQVAE  # noqa: F401
    for q in m.rq.vq_layers[:-1]:
        q.sk_epsilon = 0.0
    out = m.get_indices_groups(torch.from_numpy(x[rows]).to(dev), sizes).cpu().numpy()
    loop = torch.cat([m.get_indices(torch.from_numpy(x[rows[o:o + g]]).to(dev), use_sk=True)
                      for o, g in zip(np.cumsum([0] + sizes[:-1]), sizes)]).cpu().numpy()
    assert np.array_equal(out, loop)


@pytest.mark.parametrize("in_dim,e_dim", [(1000, 32), (1024, 32), (768, 96), (768, 128), (770, 32), (392, 32)])
def test_wider_envelope_vs_oracle(dev, in_dim, e_dim, parity_log):
    """Widths the MFMA kernels do not take or MKL's order is not pinned for (in_dim > 768,
    in_dim % 4 != 0, e_dim > 64) still encode, in rq_exact's restated order bit for bit
    (parity against the reference itself is pinned only where gr_mkl_plan says)."""
    from gr_amd import RQVAE
    torch.manual_seed(in_dim + e_dim)
    m = RQVAE(in_dim=in_dim, num_emb_list=[256, 256, 256], e_dim=e_dim, layers=[256, 128],
              sk_epsilons=[0.0] * 3).eval()
    rng = np.random.default_rng(in_dim)
    n = 600
    x = rng.standard_normal((n, in_dim), dtype=np.float32)
    lin = m.encoder.linears()
    ws = [l.weight.detach().numpy() for l in lin]
    bs = [l.bias.detach().numpy() for l in lin]
    z = rq_exact.mlp(x, ws, bs)
    with torch.no_grad():   # data-derived codebooks (codes near real latents)
        for q in m.rq.vq_layers:
            q.embedding.weight.copy_(torch.from_numpy(z[rng.integers(0, n, 256)] + 0.05 * z.std()
                                                      * rng.standard_normal((256, e_dim), dtype=np.float32)))
    cbs = [q.embedding.weight.detach().numpy() for q in m.rq.vq_layers]
    m = m.to(dev)
    xg = torch.from_numpy(x).to(dev)
    rows = differ = 0
    for M in (1, 3, 16, n):
        ref = rq_exact.encode(x[:M], ws, bs, cbs)
        got = m.get_indices(xg[:M]).cpu().numpy()
        differ += int((got != ref).any(1).sum())
        rows += M
    parity_log(kind="rq_wide_envelope", in_dim=in_dim, e_dim=e_dim, rows=rows, rows_differ=differ,
               pinned_at_600=m.parity_pinned(n))
    assert differ == 0


def test_frozen_pack_sees_graph_replayed_updates(dev):
    """a captured AdamW step changes the encoder weights without a version bump;
    get_indices must encode with the new weights (the cached image, the default, re-packs on the
    replay epoch; freeze_encoder(False) packs per call).  Also a write through .data followed by
    ops.weights_changed()."""
    from gr_amd import RQVAE, ops
    torch.manual_seed(0)
    m = RQVAE(in_dim=768, num_emb_list=[256] * 3, e_dim=32, layers=[256, 128], dropout_prob=0.0,
              sk_epsilons=[0.0] * 3).to(dev)
    opt = torch.optim.AdamW(m.parameters(), lr=torch.tensor(1e-2, device=dev), capturable=True)
    xb = torch.randn(64, 768, device=dev)
    step = ops.RqTrainGraph(m, opt, xb.clone())
    xt = torch.randn(300, 768, device=dev)
    for frozen in (False, True):
        m.freeze_encoder(frozen)
        m.eval()
        m.get_indices(xt)           # builds (and, frozen, packs) the cached binding
        m.train()
        for _ in range(3):
            step.replay()
        m.eval()
        lin = m.encoder.linears()
        ref = ops.rq_encode(xt, [l.weight.detach().clone() for l in lin], [l.bias.detach().clone() for l in lin],
                            [c.clone() for c in m.rq.codebooks()])
        assert torch.equal(m.get_indices(xt), ref), f"frozen={frozen}"
    m.freeze_encoder(True)
    m.get_indices(xt)
    lin = m.encoder.linears()
    lin[0].weight.data.mul_(0.5)    # bypasses the version counter the autograd tensor carries
    ops.weights_changed()
    ref = ops.rq_encode(xt, [l.weight.detach().clone() for l in lin], [l.bias.detach().clone() for l in lin],
                        [c.clone() for c in m.rq.codebooks()])
    assert torch.equal(m.get_indices(xt), ref)
