"""RQ-VAE encode on the GPU vs the reference's golden vectors and the CPU oracle.

Parity bar (north_star): semantic IDs bit-exact.  fp32 distances computed with a different (but
equally valid) accumulation order than the reference's CPU MKL run can only flip a row whose
best/second-best distance gap is within fp32 rounding; such rows are reported and must be
certified near-ties (gr_amd.rqvae.near_tie_rows on the reference's own distances), every other
row must be identical.
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import rq_oracle

pytestmark = pytest.mark.gpu
RQ = ["rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256"]


@pytest.fixture(params=[1, 0], ids=["fused", "layerwise"])
def rq_path(request):
    """Run a test through the fused persistent kernel and through the layer-wise path
    (gr_linear + gr_rq_quantize): both must meet the same bar."""
    from gr_amd import _lib
    _lib.set_option("rq_fused", request.param)
    yield request.param
    _lib.set_option("rq_fused", 1)


def build_model(meta, sd, dev):
    from gr_amd import RQVAE
    m = RQVAE(in_dim=meta["in_dim"], num_emb_list=[meta["K"]] * meta["L"], e_dim=meta["e_dim"],
              layers=meta["layers"], dropout_prob=0.1, sk_epsilons=[0.01] * meta["L"])
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all(k.startswith("decoder.") for k in missing)
    return m.to(dev).eval()


def near_tie_rows(out):
    """The product's own certificate (gr_amd.rqvae.near_tie_rows) on the reference's fp32 distances."""
    from gr_amd.rqvae import near_tie_rows as cert
    return cert(out["dbest"], out["gap"], out["znorm"])


# Cap on rows that may differ from the reference per fixture (every such row must also be a
# certified near-tie).  Measured on MI355X (profiles/r02_parity_counts.json): 0 / 80, 0 / 8192,
# 2 / 8192 and 0 / 2048 rows differ on both kernel paths; the caps leave room for two more rows
# where the fixture has differing rows at all.  rq_syn_randinit_3x256 is the reference's own
# uniform(+-1/K) init, the near-tie stress case (exact reference ties, gap 0.0, in 106 rows).
DIFF_CAP = {"rq_csv_3x8": 0, "rq_syn_3x256": 2, "rq_syn_4x1024": 4, "rq_syn_randinit_3x256": 2}


@pytest.mark.parametrize("name", RQ)
def test_get_indices_matches_reference(name, dev, rq_path, parity_log):
    x, sd, out, meta = gl.rq_inputs(name)
    m = build_model(meta, sd, dev)
    xg = torch.from_numpy(x).to(dev)
    idx = m.get_indices(xg).cpu().numpy()
    ref = out["idx_full"]
    assert idx.shape == ref.shape and idx.dtype == np.int64
    diff = (idx != ref).any(1)
    tie = near_tie_rows(out)
    # the product's own certificate (from the GPU's distances) flags every row that differs
    idx2, flags = m.get_indices_certified(xg)
    flags = flags.cpu().numpy()
    idx64 = torch.cat([m.get_indices(xg[i:i + 64]) for i in range(0, len(xg), 64)]).cpu().numpy()
    parity_log(kind="rq_ids", fixture=name, path="fused" if rq_path else "layerwise", rows=len(diff),
               rows_differ=int(diff.sum()), rows_ref_neartie=int(tie.sum()),
               rows_product_flagged=int(flags.sum()), rows_differ_unflagged=int((diff & ~flags).sum()),
               rows_differ_not_ref_neartie=int((diff & ~tie).sum()), cap=DIFF_CAP[name],
               batch64_rows_differ_from_full=int((idx64 != idx).any(1).sum()))
    assert not (diff & ~tie).any(), f"non-near-tie rows differ: {np.nonzero(diff & ~tie)[0][:10]}"
    assert diff.sum() <= DIFF_CAP[name]
    assert np.array_equal(idx2.cpu().numpy(), idx)
    assert not (diff & ~flags).any()
    # the batch-64 call pattern of RQ-VAE/infer.py:84-95 gives the same IDs as one batch
    assert np.array_equal(idx64, idx)


def test_quantize_on_reference_latents(dev, parity_log):
    """Given the reference's own encoder output bits, only the distance reduction order differs."""
    from gr_amd import ops
    x, sd, out, meta = gl.rq_inputs("rq_syn_3x256")
    cbs = [torch.from_numpy(sd[f"rq.vq_layers.{l}.embedding.weight"]).to(dev) for l in range(meta["L"])]
    idx, best, gap = ops.rq_quantize(torch.from_numpy(out["z"]).to(dev), cbs, with_gap=True)
    diff = (idx.cpu().numpy() != out["idx_full"]).any(1)
    tie = near_tie_rows(out)
    parity_log(kind="rq_quantize_on_ref_z", fixture="rq_syn_3x256", rows=len(diff),
               rows_differ=int(diff.sum()), rows_ref_neartie=int(tie.sum()))
    assert not (diff & ~tie).any()
    assert diff.sum() <= 2
    g = gap.cpu().numpy()
    assert (g >= 0).all()
    # the kernel's best distance and gap are the reference's fp32 values up to rounding
    np.testing.assert_allclose(best.cpu().numpy(), out["dbest"], rtol=0, atol=1e-5 * out["znorm"].max())
    np.testing.assert_allclose(g[~diff], out["gap"][~diff], rtol=0, atol=1e-5 * out["znorm"].max())


def test_encoder_latents_close_to_reference(dev, rq_path, parity_log):
    from gr_amd import ops
    x, sd, out, meta = gl.rq_inputs("rq_syn_3x256")
    m = build_model(meta, sd, dev)
    lin = m.encoder.linears()
    idx, z = ops.rq_encode(torch.from_numpy(x).to(dev), [l.weight for l in lin], [l.bias for l in lin],
                           m.rq.codebooks(), with_z=True)
    zr = out["z"]
    err = np.abs(z.cpu().numpy() - zr).max() / np.abs(zr).max()
    assert err < 1e-5, err
    from gr_amd.rqvae import Z_TAU
    row = np.linalg.norm(z.cpu().numpy().astype(np.float64) - zr, axis=1) / np.linalg.norm(zr, axis=1)
    parity_log(kind="z_tau_out_of_sample", fixture="rq_syn_3x256", path="fused" if rq_path else "layerwise",
               rows=len(row), max_row_ratio=float(row.max()), median_row_ratio=float(np.median(row)), z_tau=Z_TAU)
    assert row.max() <= Z_TAU
    # the encoder alone through the drop-in module (layer-wise kernels)
    z2 = m.encoder(torch.from_numpy(x).to(dev)).cpu().numpy()
    if rq_path == 0:
        assert np.array_equal(z2, z.cpu().numpy())
    else:
        assert np.abs(z2 - zr).max() / np.abs(zr).max() < 1e-5


def _random_case(n, e, Ks, layers, seed, dev):
    g = torch.Generator().manual_seed(seed)
    c = np.load(gl.os.path.join(gl.HERE, "csv_bert.npz"))
    x, _ = gl.synth_items(n, c["mu"], c["sigma"], seed)
    from gr_amd import RQVAE
    torch.manual_seed(seed)
    m = RQVAE(in_dim=768, num_emb_list=Ks, e_dim=e, layers=layers, sk_epsilons=[0.0] * len(Ks)).eval()
    xt = torch.from_numpy(x)
    with torch.no_grad():
        for lin in m.encoder.linears():
            lin.bias.copy_(0.01 * torch.randn(lin.bias.shape, generator=g))
        lin = m.encoder.linears()
        r = rq_oracle.mlp_encode(xt, [l.weight for l in lin], [l.bias for l in lin])
        for q in m.rq.vq_layers:   # data-derived codebooks (possibly K > n: sample with replacement)
            pick = torch.randint(0, n, (q.n_e,), generator=g)
            q.embedding.weight.copy_(r[pick] + 0.01 * r.std() * torch.randn(q.embedding.weight.shape, generator=g))
            xq, ind, _ = rq_oracle.vq_level(r, q.embedding.weight)
            r = r - xq
    ws = [l.weight.detach() for l in m.encoder.linears()]
    bs = [l.bias.detach() for l in m.encoder.linears()]
    cbs = m.rq.codebooks()
    z = rq_oracle.mlp_encode(xt, ws, bs)
    ref, residuals, gaps = rq_oracle.rq_quantize(z, cbs, return_detail=True)
    dbest = torch.stack([rq_oracle.vq_level(r, c)[2].min(1).values for r, c in zip(residuals, cbs)], -1)
    tie = near_tie_rows({"dbest": dbest.numpy(), "gap": gaps.numpy(), "znorm": (z ** 2).sum(1).numpy()})
    return m.to(dev), xt.to(dev), ref.numpy(), tie


@pytest.mark.parametrize("n,e,Ks,layers", [
    (1, 32, [8, 8, 8], [256, 128]),          # single item
    (129, 32, [256, 256, 256], [256, 128]),  # ragged last workgroup
    (1000, 32, [1024, 1, 33, 5], [256, 128]),  # fused kernel: K=1, K not a multiple of 32
    (257, 32, [16] * 8, [256, 128]),         # fused kernel: L = 8
    (500, 16, [300, 7], [64]),               # K not a multiple of 32, K > LDS chunk, e = 16
    (700, 64, [1024, 1, 33, 5], [512, 256, 128]),  # K = 1 (single code), e = 64, reference-default dims
    (333, 32, [16] * 8, [128]),              # L = 8 levels (GR_MAX_LEVELS)
])
def test_edge_shapes_vs_oracle(n, e, Ks, layers, dev, rq_path, parity_log):
    m, x, ref, tie = _random_case(n, e, Ks, layers, seed=n + e, dev=dev)
    idx = m.get_indices(x).cpu().numpy()
    diff = (idx != ref).any(1)
    parity_log(kind="rq_ids_vs_oracle", shape=f"n{n} e{e} K{Ks} layers{layers}",
               path="fused" if rq_path else "layerwise", rows=n, rows_differ=int(diff.sum()),
               rows_oracle_neartie=int(tie.sum()))
    assert not (diff & ~tie).any()
    assert (idx >= 0).all() and (idx < np.array(Ks)[None, :]).all()


def test_empty_batch(dev):
    x, sd, out, meta = gl.rq_inputs("rq_csv_3x8")
    m = build_model(meta, sd, dev)
    idx = m.get_indices(torch.zeros((0, 768), device=dev))
    assert idx.shape == (0, 3) and idx.dtype == torch.int64


def _oracle_sample(a, x_rows, m, sample):
    """(rows that differ from the oracle, oracle-side near-ties) on ``sample`` rows."""
    lin = m.encoder.linears()
    ws = [l.weight.detach().cpu() for l in lin]
    bs = [l.bias.detach().cpu() for l in lin]
    cbs = [q.cpu() for q in m.rq.codebooks()]
    zs = rq_oracle.mlp_encode(x_rows, ws, bs)
    ref, res, gaps = rq_oracle.rq_quantize(zs, cbs, return_detail=True)
    dbest = torch.stack([rq_oracle.vq_level(r, c)[2].min(1).values for r, c in zip(res, cbs)], -1)
    diff = (a[sample.to(a.device)].cpu().numpy() != ref.numpy()).any(1)
    tie = near_tie_rows({"dbest": dbest.numpy(), "gap": gaps.numpy(), "znorm": (zs ** 2).sum(1).numpy()})
    return diff, tie


def test_full_size_c2_properties(dev, rq_path, parity_log):
    """Config 2 size (100k items, 3x256): determinism, range, agreement with the oracle on a sample,
    and self-consistency of the two entry points (encode == quantize(encoder(x)))."""
    from gr_amd import ops
    m, _, _, _ = _random_case(64, 32, [256] * 3, [256, 128], seed=5, dev=dev)
    c = np.load(gl.os.path.join(gl.HERE, "csv_bert.npz"))
    x, _ = gl.synth_items(100_000, c["mu"], c["sigma"], 99)
    xg = torch.from_numpy(x).to(dev)
    a = m.get_indices(xg)
    b = m.get_indices(xg)
    assert torch.equal(a, b)
    assert int(a.min()) >= 0 and int(a.max()) < 256
    lin = m.encoder.linears()
    idx_z, z = ops.rq_encode(xg, [l.weight for l in lin], [l.bias for l in lin], m.rq.codebooks(),
                             with_z=True)
    assert torch.equal(idx_z, a)
    q = ops.rq_quantize(z, m.rq.codebooks())   # the standalone quantizer on the same latents
    # ||r||^2 is summed in a different order by the two kernels: only near-ties may move
    n_q = (q != a).any(1).sum().item()
    sample = torch.arange(0, 100_000, 49)
    diff, tie = _oracle_sample(a, torch.from_numpy(x[sample.numpy()]), m, sample)
    _, flags = m.get_indices_certified(xg)
    parity_log(kind="rq_ids_full_size", config="C2-shape (64-row codebooks)", path="fused" if rq_path else "layerwise",
               rows=100_000, rows_product_flagged=int(flags.sum()), oracle_sample_rows=len(sample),
               oracle_sample_rows_differ=int(diff.sum()), oracle_sample_rows_neartie=int(tie.sum()),
               quantize_vs_encode_rows_differ=n_q)
    assert n_q <= 100
    assert not (diff & ~tie).any()


def test_full_size_c2_bench_workload(dev, rq_path, parity_log):
    """The exact C2 bench workload (synth.rqvae_model(3, 256), synth.items(100k, seed 1000)):
    oracle agreement on 2041 strided rows + the last 64, and the product certificate's flag count
    over all 100k rows ("report the near-tie fallback count")."""
    from gr_amd import synth
    n = 100_000
    m = synth.rqvae_model(3, 256, dev)
    x = synth.items(n, 1000, dev)
    a = m.get_indices(x)
    idx2, flags = m.get_indices_certified(x)
    assert torch.equal(idx2, a)
    sample = torch.cat([torch.arange(0, n, 49), torch.arange(n - 64, n)])
    diff, tie = _oracle_sample(a, x[sample.to(dev)].cpu(), m, sample)
    fl = flags[sample.to(dev)].cpu().numpy()
    parity_log(kind="rq_ids_full_size", config="C2 bench workload", path="fused" if rq_path else "layerwise",
               rows=n, rows_product_flagged=int(flags.sum()), oracle_sample_rows=len(sample),
               oracle_sample_rows_differ=int(diff.sum()), oracle_sample_rows_neartie=int(tie.sum()),
               oracle_sample_rows_differ_unflagged=int((diff & ~fl).sum()))
    assert not (diff & ~tie).any()
    assert not (diff & ~fl).any()


def test_full_size_c4_properties(dev, rq_path, parity_log):
    """Config 4 size (10M items, 4x1024 codebooks, 30.7 GB of input in HBM): the input spans
    7.68e9 floats, so rows past 2^31 elements exercise 64-bit addressing.  Range, determinism, and
    agreement with the oracle on a strided sample plus the last 64 rows (near-ties excepted); the
    product certificate's flag count over all 10M rows."""
    from gr_amd import synth
    n = 10_000_000
    m = synth.rqvae_model(4, 1024, dev, seed=4)
    x = synth.items(n, 4000, dev)
    a = m.get_indices(x)
    assert a.shape == (n, 4) and a.dtype == torch.int64
    assert int(a.min()) >= 0 and int(a.max()) < 1024
    tail = slice(n - 4096, n)
    # the same rows re-encoded as their own batch (offset 0): only batch-size-dependent launch
    # plans may differ, and those only on near-ties
    n_tail = (m.get_indices(x[tail]) != a[tail]).any(1).sum().item()
    sample = torch.cat([torch.arange(0, n, 5003), torch.arange(n - 64, n)])
    xs = x[sample.to(dev)].cpu()
    idx2, flags = m.get_indices_certified(x)
    assert torch.equal(idx2, a)
    n_flag = int(flags.sum())
    fl = flags[sample.to(dev)].cpu().numpy()
    del x, idx2, flags
    diff, tie = _oracle_sample(a, xs, m, sample)
    parity_log(kind="rq_ids_full_size", config="C4 (10M x 4x1024)", path="fused" if rq_path else "layerwise",
               rows=n, rows_product_flagged=n_flag, oracle_sample_rows=len(sample),
               oracle_sample_rows_differ=int(diff.sum()), oracle_sample_rows_neartie=int(tie.sum()),
               oracle_sample_rows_differ_unflagged=int((diff & ~fl).sum()),
               tail_rebatch_rows_differ=n_tail)
    assert n_tail <= 4
    assert not (diff & ~tie).any()
    assert not (diff & ~fl).any()


def test_binding_cache_sees_weight_changes(dev):
    """The cached pointer view (ops.rq_binding) follows in-place updates (load_state_dict) and
    storage swaps (param.data = ...): results always equal a fresh uncached encode."""
    from gr_amd import ops
    x, sd, out, meta = gl.rq_inputs("rq_syn_3x256")
    m = build_model(meta, sd, dev)
    xg = torch.from_numpy(x[:512]).to(dev)

    def fresh():
        lin = m.encoder.linears()
        return ops.rq_encode(xg, [l.weight for l in lin], [l.bias for l in lin], m.rq.codebooks())
    a = m.get_indices(xg)
    assert m.encode_binding() is m.encode_binding()
    sd2 = {k: v.clone() for k, v in m.state_dict().items()}
    sd2["rq.vq_layers.0.embedding.weight"] = sd2["rq.vq_layers.0.embedding.weight"].flip(0)
    m.load_state_dict(sd2)                                   # in place: same pointers
    b = m.get_indices(xg)
    assert torch.equal(b, fresh()) and not torch.equal(a, b)
    w = m.rq.vq_layers[0].embedding.weight
    w.data = w.data.flip(0).clone()                           # new storage
    c = m.get_indices(xg)
    assert torch.equal(c, fresh()) and torch.equal(c, a)


def test_batchnorm_encoder_matches_reference(dev, rq_path, parity_log):
    """RQVAE(bn=True) (RQ-VAE/models/layers.py:25-26) in eval mode: the BatchNorm folds into its
    Linear; IDs equal the reference's except certified near-ties (tests/golden/make_golden_bn.py)."""
    from gr_amd import RQVAE
    x, sd, out, meta = gl.rq_inputs("rq_bn_3x256")
    m = RQVAE(in_dim=768, num_emb_list=[meta["K"]] * meta["L"], e_dim=32, layers=[256, 128], dropout_prob=0.1,
              bn=True, sk_epsilons=[0.0] * meta["L"])
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all(k.startswith("decoder.") for k in missing)
    m = m.to(dev).eval()
    xg = torch.from_numpy(x).to(dev)
    idx = m.get_indices(xg).cpu().numpy()
    diff = (idx != out["idx_full"]).any(1)
    tie = near_tie_rows(out)
    _, flags = m.get_indices_certified(xg)
    flags = flags.cpu().numpy()
    z = m.encoder(xg).cpu().numpy()
    zerr = (np.linalg.norm(z.astype(np.float64) - out["z"], axis=1) / np.linalg.norm(out["z"], axis=1)).max()
    parity_log(kind="rq_ids", fixture="rq_bn_3x256", path="fused" if rq_path else "layerwise", rows=len(diff),
               rows_differ=int(diff.sum()), rows_ref_neartie=int(tie.sum()), rows_product_flagged=int(flags.sum()),
               max_row_z_ratio=float(zerr))
    assert not (diff & ~tie).any() and not (diff & ~flags).any()
    assert diff.sum() <= 2
    from gr_amd.rqvae import Z_TAU
    assert zerr <= Z_TAU


@pytest.mark.parametrize("act", ["sigmoid", "tanh", "leakyrelu", "none", "relu"])
@pytest.mark.parametrize("bn", [False, True])
def test_mlp_activations_and_batchnorm_vs_torch(act, bn, dev):
    """MLPLayers with every activation of RQ-VAE/models/layers.py:45-67 and optional BatchNorm, eval
    mode, against the same module tree run by torch on the CPU (fp32, 1e-5 relative)."""
    from gr_amd.rqvae import MLPLayers
    torch.manual_seed(7)
    m = MLPLayers([96, 64, 48, 16], dropout=0.1, activation=act, bn=bn)
    with torch.no_grad():
        for mod in m.mlp_layers:
            if isinstance(mod, torch.nn.BatchNorm1d):
                mod.running_mean.normal_(0, 0.3)
                mod.running_var.uniform_(0.5, 2.0)
                mod.weight.normal_(1, 0.1)
                mod.bias.normal_(0, 0.1)
    m.eval()
    x = torch.randn(300, 96)
    with torch.no_grad():
        ref = m.mlp_layers(x)
    mg = m.to(dev)
    with torch.no_grad():
        got = mg(x.to(dev)).cpu()
        got2 = mg.eval_forward(x.to(dev)).cpu()
    scale = ref.abs().max()
    assert (got - ref).abs().max() <= 1e-5 * scale
    assert (got2 - ref).abs().max() <= 1e-5 * scale
