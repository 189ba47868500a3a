"""RQ-VAE encode on the GPU vs the reference's golden vectors and the exact-order CPU oracle.

Parity bar (north_star): semantic IDs bit-exact.  The kernels compute in the reference's own CPU
summation order (oracle/rq_exact.c, pinned against every fixture by tests/test_rq_exact_oracle.py),
so every row must be identical -- exact fp32 ties included -- on both encoder paths (the fused
persistent kernel and the layer-wise exact gr_linear path), at fixture size and over whole C2 / C4
populations.
"""
import numpy as np
import pytest
import torch

import golden_lib as gl
from oracle import rq_exact

pytestmark = pytest.mark.gpu
RQ = ["rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256", "rq_calib_3x256",
      "rq_calib_wide_3x256"]


@pytest.fixture(params=[1, 0], ids=["fused", "layerwise"])
def rq_path(request):
    """Run a test through the fused persistent kernel and through the layer-wise path
    (exact gr_linear + gr_rq_quantize): both must be bitwise the reference."""
    from gr_amd import _lib
    _lib.set_option("rq_fused", request.param)
    yield request.param
    _lib.set_option("rq_fused", 1)


def build_model(meta, sd, dev, bn=False):
    from gr_amd import RQVAE
    m = RQVAE(in_dim=meta["in_dim"] if "in_dim" in meta else 768, num_emb_list=[meta["K"]] * meta["L"],
              e_dim=meta["e_dim"], layers=meta["layers"], dropout_prob=0.1, bn=bn,
              sk_epsilons=[0.01] * meta["L"])
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert not unexpected and all(k.startswith("decoder.") for k in missing)
    return m.to(dev).eval()


def _path(p):
    return "fused" if p else "layerwise"


@pytest.mark.parametrize("name", RQ)
def test_get_indices_matches_reference(name, dev, rq_path, parity_log):
    x, sd, out, meta = gl.rq_inputs(name)
    m = build_model(meta, sd, dev)
    xg = torch.from_numpy(x).to(dev)
    idx = m.get_indices(xg).cpu().numpy()
    ref = out["idx_full"]
    assert idx.shape == ref.shape and idx.dtype == np.int64
    diff = (idx != ref).any(1)
    # the batch-64 call pattern of RQ-VAE/infer.py:84-95 gives the same IDs as one batch
    idx64 = torch.cat([m.get_indices(xg[i:i + 64]) for i in range(0, len(xg), 64)]).cpu().numpy()
    lin = m.encoder.linears()
    from gr_amd import ops
    _, z = ops.rq_encode(xg, [l.weight for l in lin], [l.bias for l in lin], m.rq.codebooks(), with_z=True)
    z = z.cpu().numpy()
    zref = out["z"] if "z" in out else rq_exact.mlp(x, [l.weight.detach().cpu() for l in lin],
                                                    [l.bias.detach().cpu() for l in lin])
    parity_log(kind="rq_ids", fixture=name, path=_path(rq_path), rows=len(diff), rows_differ=int(diff.sum()),
               z_rows_differ=int((z != zref).any(1).sum()),
               batch64_rows_differ_from_full=int((idx64 != idx).any(1).sum()))
    assert diff.sum() == 0, f"rows differ from the reference: {np.nonzero(diff)[0][:10]}"
    assert np.array_equal(z, zref), "encoder output is not the reference's bits"
    assert np.array_equal(idx64, idx)


@pytest.mark.parametrize("name", ["rq_syn_3x256", "rq_calib_3x256", "rq_calib_wide_3x256", "rq_bn_3x256"])
def test_quantize_on_reference_latents(name, dev, parity_log):
    """The quantizer alone on the reference's own encoder output bits: exact, best distance and gap
    equal to the exact-order oracle's."""
    from gr_amd import ops
    x, sd, out, meta = gl.rq_inputs(name)
    cbs = [sd[f"rq.vq_layers.{l}.embedding.weight"] for l in range(meta["L"])]
    idx, best, gap = ops.rq_quantize(torch.from_numpy(out["z"]).to(dev), [torch.from_numpy(c).to(dev) for c in cbs],
                                     with_gap=True)
    ridx, rbest, rgap = rq_exact.quantize(out["z"], cbs, with_detail=True)
    diff = (idx.cpu().numpy() != out["idx_full"]).any(1)
    parity_log(kind="rq_quantize_on_ref_z", fixture=name, rows=len(diff), rows_differ=int(diff.sum()))
    assert diff.sum() == 0
    assert np.array_equal(ridx, out["idx_full"])
    assert np.array_equal(best.cpu().numpy(), rbest)
    assert np.array_equal(gap.cpu().numpy(), rgap)


def _random_case(n, e, Ks, layers, seed, dev):
    """Random RQ-VAE with data-derived codebooks: distinct residual rows plus noise (K <= n), or
    Gaussian codes at the residuals' scale (K > n), so the code sets are never degenerate."""
    from gr_amd import RQVAE
    g = torch.Generator().manual_seed(seed)
    c = np.load(gl.os.path.join(gl.HERE, "csv_bert.npz"))
    x, _ = gl.synth_items(n, c["mu"], c["sigma"], seed)
    torch.manual_seed(seed)
    m = RQVAE(in_dim=768, num_emb_list=Ks, e_dim=e, layers=layers, sk_epsilons=[0.0] * len(Ks)).eval()
    with torch.no_grad():
        for lin in m.encoder.linears():
            lin.bias.copy_(0.01 * torch.randn(lin.bias.shape, generator=g))
        lin = m.encoder.linears()
        r = torch.from_numpy(rq_exact.mlp(x, [l.weight.detach() for l in lin], [l.bias.detach() for l in lin]))
        for q in m.rq.vq_layers:
            if q.n_e <= n:
                pick = torch.randperm(n, generator=g)[:q.n_e]
                cb = r[pick] + 0.01 * r.std() * torch.randn(q.embedding.weight.shape, generator=g)
            else:
                cb = r.mean(0) + r.std(0) * torch.randn(q.embedding.weight.shape, generator=g)
            q.embedding.weight.copy_(cb)
            idx = torch.from_numpy(rq_exact.quantize(r.numpy(), [cb.numpy()])[:, 0])
            cq = cb[idx]
            r = r - (r + (cq - r))
    ws = [l.weight.detach() for l in m.encoder.linears()]
    bs = [l.bias.detach() for l in m.encoder.linears()]
    ref = rq_exact.encode(x, ws, bs, m.rq.codebooks())
    return m.to(dev), torch.from_numpy(x).to(dev), ref


@pytest.mark.parametrize("n,e,Ks,layers", [
    (1, 32, [8, 8, 8], [256, 128]),          # single item
    (129, 32, [256, 256, 256], [256, 128]),  # ragged last workgroup
    (1000, 32, [1024, 1, 33, 5], [256, 128]),  # fused kernel: K=1, K not a multiple of 32, K > n
    (257, 32, [16] * 8, [256, 128]),         # fused kernel: L = 8
    (500, 16, [300, 7], [64]),               # K not a multiple of 32, e = 16
    (700, 64, [1024, 1, 33, 5], [512, 256, 128]),  # K = 1, e = 64, rqvae.py's default widths, K > n
    (333, 32, [16] * 8, [128]),              # L = 8 levels (GR_MAX_LEVELS)
    (600, 20, [64, 64, 64], [256, 128]),     # e not a multiple of 8 (zero-padded features)
    (400, 8, [32, 32], [128]),               # e = 8
    (300, 48, [128, 128], [512, 256]),       # e = 48, two-block first layer on the layer-wise path
    (250, 5, [16, 16, 16], [64]),            # e < 8: ATen's scalar row sum
    (5000, 64, [256, 256], [256, 128]),      # e = 64 over several tiles per wave
])
def test_edge_shapes_vs_oracle(n, e, Ks, layers, dev, rq_path, parity_log):
    m, x, ref = _random_case(n, e, Ks, layers, seed=n + e, dev=dev)
    idx = m.get_indices(x).cpu().numpy()
    diff = (idx != ref).any(1)
    parity_log(kind="rq_ids_vs_oracle", shape=f"n{n} e{e} K{Ks} layers{layers}", path=_path(rq_path),
               rows=n, rows_differ=int(diff.sum()))
    assert diff.sum() == 0
    assert (idx >= 0).all() and (idx < np.array(Ks)[None, :]).all()


def test_empty_batch(dev):
    x, sd, out, meta = gl.rq_inputs("rq_csv_3x8")
    m = build_model(meta, sd, dev)
    idx = m.get_indices(torch.zeros((0, 768), device=dev))
    assert idx.shape == (0, 3) and idx.dtype == torch.int64


def _weights(m):
    lin = m.encoder.linears()
    return ([l.weight.detach().cpu() for l in lin], [l.bias.detach().cpu() for l in lin],
            [c.cpu() for c in m.rq.codebooks()])


def test_full_population_c2_bench_workload(dev, rq_path, parity_log):
    """The exact C2 bench workload (synth.rqvae_model(3, 256), synth.items(100k, seed 1000)): ALL
    100,000 rows against the exact-order oracle."""
    from gr_amd import synth
    n = 100_000
    m = synth.rqvae_model(3, 256, dev)
    x = synth.items(n, 1000, dev)
    a = m.get_indices(x)
    assert torch.equal(a, m.get_indices(x))
    ws, bs, cbs = _weights(m)
    ref = rq_exact.encode(x.cpu().numpy(), ws, bs, cbs)
    diff = (a.cpu().numpy() != ref).any(1)
    parity_log(kind="rq_ids_full_population", config="C2 bench workload", path=_path(rq_path), rows=n,
               rows_differ=int(diff.sum()))
    assert diff.sum() == 0, f"{diff.sum()} of {n} rows differ: {np.nonzero(diff)[0][:10]}"


@pytest.mark.parametrize("n", [1, 31, 33, 64, 255 * 32 + 7, 256 * 32, 256 * 33 + 1, 256 * 34 + 5])
def test_partition_edges_vs_oracle(n, dev, parity_log):
    """Batch sizes around the fused encoder's tile partition: fewer tiles than CUs (every workgroup
    runs ONE k-split pass -- the tile's two MKL k blocks as its two chains), an odd last tile after
    full passes, exact multiples; every row against the exact-order oracle, and back-to-back calls
    equal."""
    from gr_amd import synth
    m = synth.rqvae_model(3, 256, dev)
    x = synth.items(n, 77, dev)
    one = m.get_indices(x)
    again = [m.get_indices(x) for _ in range(4)]   # back to back, no host sync in between
    assert all(torch.equal(one, a) for a in again)
    ws, bs, cbs = _weights(m)
    ref = rq_exact.encode(x.cpu().numpy(), ws, bs, cbs)
    diff = (one.cpu().numpy() != ref).any(1)
    parity_log(kind="rq_ids_vs_oracle", shape=f"C2 model, n {n} (partition edges)", path="fused", rows=n,
               rows_differ=int(diff.sum()))
    assert diff.sum() == 0, f"{diff.sum()} of {n} rows differ"


@pytest.mark.parametrize("n,Ks", [
    (16, [256, 256, 256]), (17, [256, 256, 256]), (31, [256, 256, 256]), (33, [256, 256, 256]),
    (64, [256, 256, 256]), (100, [256, 256, 256]), (128, [256, 256, 256]), (255, [256, 256, 256]),
    (256, [256, 256, 256]), (257, [256, 256, 256]), (1000, [256, 256, 256]), (1024, [256, 256, 256]),
    (1025, [256, 256, 256]), (64, [1, 33, 5, 512]), (48, [16] * 8), (200, [500, 7]),
])
def test_short_call_kernels_vs_oracle(n, Ks, dev, parity_log):
    """Calls of 16-1024 rows (the reference's batch of 64) run on the short-call kernels
    (rq_small.hip: 16x16x4 chains, layer 1 over 16 feature tiles and layer 2 over 8 per 16 rows,
    then layer 3 and every quantizer level in one workgroup per 16 rows): IDs and z against the
    exact-order oracle, codebooks of 1..512 codes (K not a multiple of 16) and 8 levels; 1025 rows
    take the long-call kernels."""
    from gr_amd import ops
    m, x, ref = _random_case(n, 32, Ks, [256, 128], seed=3 * n + len(Ks), dev=dev)
    idx = m.get_indices(x).cpu().numpy()
    lin = m.encoder.linears()
    idx2, z = ops.rq_encode(x, [l.weight for l in lin], [l.bias for l in lin], m.rq.codebooks(), with_z=True)
    zref = rq_exact.mlp(x.cpu().numpy(), [l.weight.detach().cpu() for l in lin], [l.bias.detach().cpu() for l in lin])
    diff = (idx != ref).any(1)
    parity_log(kind="rq_ids_vs_oracle", shape=f"short call n {n} K{Ks}", path="fused", rows=n,
               rows_differ=int(diff.sum()), z_rows_differ=int((z.cpu().numpy() != zref).any(1).sum()))
    assert diff.sum() == 0, f"{diff.sum()} of {n} rows differ"
    assert np.array_equal(idx2.cpu().numpy(), idx)
    assert np.array_equal(z.cpu().numpy(), zref)


def test_full_population_c4_contiguous(dev, parity_log):
    """Config 4 size (10M items, 4x1024 codebooks, 30.7 GB of input in HBM; rows past 2^31 floats
    exercise 64-bit addressing): the 10M-row encode checked against the exact-order oracle on the
    first 1,048,576 contiguous rows (whole workgroup ranges: 3,815 workgroups of 32 tiles) and the
    last 65,536 rows."""
    from gr_amd import synth
    n = 10_000_000
    m = synth.rqvae_model(4, 1024, dev, seed=4)
    x = synth.items(n, 4000, dev)
    a = m.get_indices(x)
    assert a.shape == (n, 4) and a.dtype == torch.int64
    assert int(a.min()) >= 0 and int(a.max()) < 1024
    ws, bs, cbs = _weights(m)
    head, tail = slice(0, 1 << 20), slice(n - 65536, n)
    xh, xt = x[head].cpu().numpy(), x[tail].cpu().numpy()
    ah, at = a[head].cpu().numpy(), a[tail].cpu().numpy()
    del x, a
    torch.cuda.empty_cache()
    dh = (ah != rq_exact.encode(xh, ws, bs, cbs)).any(1)
    dt = (at != rq_exact.encode(xt, ws, bs, cbs)).any(1)
    parity_log(kind="rq_ids_full_population", config="C4 (10M x 4x1024), rows [0, 2^20) + last 65536",
               path="fused", rows=int(len(dh) + len(dt)), rows_differ=int(dh.sum() + dt.sum()))
    assert dh.sum() == 0 and dt.sum() == 0, (int(dh.sum()), int(dt.sum()))


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
    sd2["encoder.mlp_layers.1.weight"] = sd2["encoder.mlp_layers.1.weight"] * 1.5
    m.load_state_dict(sd2)                                   # in place: same pointers
    b = m.get_indices(xg)
    assert torch.equal(b, fresh()) and not torch.equal(a, b)
    w = m.rq.vq_layers[0].embedding.weight
    w.data = w.data.flip(0).clone()                           # new storage
    c = m.get_indices(xg)
    assert torch.equal(c, fresh())


def test_batchnorm_encoder_matches_reference(dev, rq_path, parity_log):
    """RQVAE(bn=True) (RQ-VAE/models/layers.py:25-26) in eval mode: the BatchNorm in torch's CPU
    formula after its Linear (not folded); z and IDs bitwise the reference's
    (tests/golden/make_golden_bn.py)."""
    x, sd, out, meta = gl.rq_inputs("rq_bn_3x256")
    m = build_model(dict(meta, e_dim=32, layers=[256, 128]), sd, dev, bn=True)
    xg = torch.from_numpy(x).to(dev)
    idx = m.get_indices(xg).cpu().numpy()
    diff = (idx != out["idx_full"]).any(1)
    z = m.encoder(xg).cpu().numpy()
    parity_log(kind="rq_ids", fixture="rq_bn_3x256", path=_path(rq_path), rows=len(diff),
               rows_differ=int(diff.sum()), z_rows_differ=int((z != out["z"]).any(1).sum()))
    assert diff.sum() == 0
    assert np.array_equal(z, out["z"])
    idx2, flags = m.get_indices_certified(xg)
    assert np.array_equal(idx2.cpu().numpy(), idx)


@pytest.mark.parametrize("act", ["leakyrelu", "none", "relu"])
@pytest.mark.parametrize("bn", [False, True])
def test_mlp_exact_activations_and_batchnorm(act, bn, dev):
    """MLPLayers with the activations torch evaluates exactly (layers.py:45-67) and optional
    BatchNorm, eval mode: bitwise the exact-order oracle (itself pinned against torch's CPU ops)."""
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
    lin = m.linears()
    bnp = None
    if bn:
        bns = [b for b in m.mlp_layers if isinstance(b, torch.nn.BatchNorm1d)]
        bnp = ([b.running_mean.numpy() for b in bns], [b.running_var.numpy() for b in bns],
               [b.weight.detach().numpy() for b in bns], [b.bias.detach().numpy() for b in bns], 1e-5)
    ref = rq_exact.mlp(x.numpy(), [l.weight.detach().numpy() for l in lin], [l.bias.detach().numpy() for l in lin],
                       bn=bnp, act=act)
    got = m.to(dev)(x.to(dev)).cpu().numpy()
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("act", ["sigmoid", "tanh"])
def test_mlp_smooth_activations_vs_torch(act, dev):
    """Sigmoid / Tanh MLPs (gr_linear_f32 epilogues): fp32-close to torch (1e-5 relative) -- torch's
    CPU exp / tanh are its own vectorised approximations, so these are not bitwise."""
    from gr_amd.rqvae import MLPLayers
    torch.manual_seed(7)
    m = MLPLayers([96, 64, 48, 16], dropout=0.1, activation=act, bn=False).eval()
    x = torch.randn(300, 96)
    with torch.no_grad():
        ref = m.mlp_layers(x)
        got = m.to(dev)(x.to(dev)).cpu()
    assert (got - ref).abs().max() <= 1e-5 * ref.abs().max()
