"""Generate the golden fixtures under tests/golden/ by running the REFERENCE itself on CPU.

Container-only: imports ``RQ-VAE/models`` and ``SASRec/model.py`` from /root/reference (read-only,
never shipped).  Only the emitted data (``*.npz``) is committed; nothing here runs on the GPU box.

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Inputs that are large (synthetic item embeddings) are not stored: they are regenerated
bit-exactly from a numpy PCG64 seed by ``golden_lib.synth_items`` and checked against a stored
SHA-256.  Everything else (state dicts, sequences, targets, expected outputs) is stored.
"""
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import golden_lib as gl  # noqa: E402
from oracle import rq_oracle, sasrec_oracle, metrics_oracle  # noqa: E402

REF = "/root/reference"
torch.set_num_threads(8)


def _import_ref():
    sys.path.insert(0, os.path.join(REF, "RQ-VAE"))
    from models.rqvae import RQVAE  # noqa
    sys.path.pop(0)
    sys.path.insert(0, os.path.join(REF, "SASRec"))
    import model as sasrec_model  # noqa
    sys.path.pop(0)
    return RQVAE, sasrec_model.SASRec


def load_csv():
    """stu-major/interaction_records.csv: the 80 rows with a student_id, in file (id) order."""
    import pandas as pd
    df = pd.read_csv(os.path.join(REF, "stu-major/interaction_records.csv"), encoding="utf-8-sig")
    df = df[df.student_id.notna()].sort_values("id")
    vecs = np.array([json.loads(s) for s in df.bert_vector], dtype=np.float64).astype(np.float32)
    return df.student_id.astype(str).tolist(), df.class_id.astype(np.int64).to_numpy(), vecs


# ----------------------------------------------------------------------------- RQ-VAE
def make_rq(RQVAE, name, x, L, K, seed, perturb_bias=True, data_codebooks=True, e_dim=32,
            layers=(256, 128)):
    torch.manual_seed(seed)
    model = RQVAE(in_dim=x.shape[1], num_emb_list=[K] * L, e_dim=e_dim, layers=list(layers),
                  dropout_prob=0.1, bn=False, loss_type="mse", quant_loss_weight=0.1, beta=0.25,
                  kmeans_init=False, kmeans_iters=50, sk_epsilons=[0.01] * L, sk_iters=50).eval()
    xt = torch.from_numpy(x)
    with torch.no_grad():
        if perturb_bias:
            g = torch.Generator().manual_seed(seed + 100)
            for m in model.encoder.mlp_layers:
                if isinstance(m, torch.nn.Linear):
                    m.bias.copy_(0.01 * torch.randn(m.bias.shape, generator=g))
        if data_codebooks:
            # level-l codebook = K residual rows (seeded randperm) + 0.01*std noise, a k-means-like init
            z = model.encoder(xt)
            r = z
            for l, vq in enumerate(model.rq.vq_layers):
                g = torch.Generator().manual_seed(seed + 1 + l)
                pick = torch.randperm(r.shape[0], generator=g)[:K]
                cb = r[pick] + 0.01 * r.std() * torch.randn((K, r.shape[1]), generator=g)
                vq.embedding.weight.copy_(cb)
                x_res, _, _ = vq(r, use_sk=False)
                r = r - x_res
        idx_full = model.get_indices(xt, use_sk=False)
        idx_b64 = torch.cat([model.get_indices(xt[i:i + 64], use_sk=False)
                             for i in range(0, xt.shape[0], 64)])
        z = model.encoder(xt)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ws, bs, cbs = rq_oracle.state_to_lists(sd, L)
    o_idx, residuals, gaps = rq_oracle.rq_quantize(rq_oracle.mlp_encode(xt, ws, bs), cbs, return_detail=True)
    assert torch.equal(o_idx, idx_full), f"{name}: oracle restatement != reference"
    # fp64 recompute, for documentation of fp32 rounding sensitivity
    i64 = rq_oracle.rq_quantize(rq_oracle.mlp_encode(xt.double(), [w.double() for w in ws],
                                                     [b.double() for b in bs]), [c.double() for c in cbs])
    rn = torch.stack([(r ** 2).sum(1) for r in residuals], -1)
    dbest = torch.stack([rq_oracle.vq_level(r, c)[2].min(1).values for r, c in zip(residuals, cbs)], -1)
    meta = dict(name=name, L=L, K=K, e_dim=e_dim, layers=list(layers), in_dim=x.shape[1], n=x.shape[0],
                seed=seed, data_codebooks=data_codebooks, torch=torch.__version__,
                fp32_vs_fp64_rows=int((i64 != idx_full).any(1).sum()),
                batch64_vs_full_rows=int((idx_b64 != idx_full).any(1).sum()))
    out = dict(idx_full=idx_full.numpy(), idx_b64=idx_b64.numpy(), z=z.numpy(),
               gap=gaps.numpy(), resid_norm=rn.numpy(),
               dbest=dbest.numpy(), znorm=(z ** 2).sum(1).numpy())
    return sd, out, meta


# ----------------------------------------------------------------------------- SASRec
def sas_params(d, n, blocks, heads, mlp, eps=1e-8):
    return {"device": "cpu", "d": d, "max_len": n, "num_blocks": blocks, "num_heads": heads,
            "dropout": 0.2, "mlp_layer": mlp, "layernorm_eps": eps}


def make_sasrec(SASRec, name, item_num, params, seqs, seed, perturb=True, target_mode="mixed",
                targets=None, n_forward=8):
    torch.manual_seed(seed)
    model = SASRec(item_num, params).eval()
    if perturb:
        g = torch.Generator().manual_seed(seed + 100)
        with torch.no_grad():
            for k, v in model.state_dict().items():
                if k.endswith("bias") or "layernorm" in k:
                    v.add_(0.05 * torch.randn(v.shape, generator=g))
    ids = torch.from_numpy(seqs)
    with torch.no_grad():
        logits = model.predict(ids)
        feats = model.forward(ids[:n_forward])
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    o_logits = sasrec_oracle.predict(ids, sd, params["num_blocks"], params["num_heads"],
                                     params["layernorm_eps"])
    bitexact = bool(torch.equal(o_logits, logits))
    if params["num_heads"] % 2 == 1:
        assert bitexact, f"{name}: oracle restatement != reference (odd heads must be bit-exact)"
    if targets is None:
        g = np.random.default_rng(seed + 7)
        lg = logits.clone()
        lg[:, 0] = -1e9
        top20 = torch.topk(lg, 20, dim=1).indices.numpy()
        targets = np.where(g.random(len(seqs)) < 0.5, top20[np.arange(len(seqs)), g.integers(0, 20, len(seqs))],
                           g.integers(1, item_num + 1, len(seqs))).astype(np.int64)
    t = torch.from_numpy(targets)
    # evaluate.py:27-32 verbatim semantics
    lg = logits.clone()
    lg[:, 0] = -1e9
    ts = lg.gather(1, t.unsqueeze(1))
    ranks = ((lg > ts).sum(dim=1) + 1).numpy()
    assert np.array_equal(ranks, metrics_oracle.ranks_from_logits(logits, t).numpy())
    hr, ndcg = metrics_oracle.hr_ndcg(ranks, 10)
    # per-user certification margin: distance of the target logit to its nearest competitor
    other = lg.clone()
    other.scatter_(1, t.unsqueeze(1), float("inf"))
    margin = (other - ts).abs().min(dim=1).values / lg[:, 1:].abs().max(dim=1).values
    meta = dict(name=name, item_num=item_num, params=params, seed=seed, perturb=perturb,
                oracle_bitexact=bitexact, torch=torch.__version__, hr10=hr, ndcg10=ndcg, B=len(seqs))
    out = dict(seqs=seqs, targets=targets, logits=logits.numpy(), forward=feats.numpy(),
               ranks=ranks, margin=margin.numpy())
    return sd, out, meta


def random_seqs(rng, B, n, item_num, edge=True):
    """Test-mode sequences (SASRec/data_vision.py:74-87): history = last n of seq[:-1], left-pad 0."""
    out = np.zeros((B, n), dtype=np.int64)
    for b in range(B):
        hist = int(rng.integers(1, n + 6))      # some longer than n (truncated), some short
        items = rng.integers(1, item_num + 1, hist)
        s = items[-n:]
        out[b, n - len(s):] = s
    if edge:
        out[0] = 0                          # all-padding row (data_vision.py:74-75, len(seq) < 2)
        out[1, :] = rng.integers(1, item_num + 1, n)   # full length, no padding
        out[2, :-1] = 0                     # a single history item
        out[2, -1] = item_num               # the last catalog row
    return out


def main():
    RQVAE, SASRec = _import_ref()
    students, class_ids, vecs = load_csv()
    mu, sigma = vecs.mean(0), vecs.std(0)
    np.savez_compressed(os.path.join(HERE, "csv_bert.npz"), vecs=vecs, class_id=class_ids,
                        student_id=np.array(students), mu=mu.astype(np.float32), sigma=sigma.astype(np.float32))
    print("csv:", vecs.shape, "mu norm", float(np.linalg.norm(mu)))

    def save(name, sd, out, meta, keep_decoder=False, keep_z=True):
        # the decoder is not on the get_indices path: keep it only where state_dict loading is tested
        arrs = {f"sd/{k}": v.numpy() for k, v in sd.items() if keep_decoder or not k.startswith("decoder.")}
        if not keep_z:
            out = {k: v for k, v in out.items() if k != "z"}
        arrs.update(out)
        arrs["meta"] = np.array(json.dumps(meta))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print(name, {k: v for k, v in meta.items() if k not in ("params",)})

    # --- RQ-VAE: config 1 data (80 real BERT vectors), main.py codebooks 3x8
    sd, out, meta = make_rq(RQVAE, "rq_csv_3x8", vecs, 3, 8, seed=0)
    save("rq_csv_3x8", sd, out, meta, keep_decoder=True)
    # --- RQ-VAE: synthetic mu+sigma*eps, C2 (3x256) and C4 (4x1024) shapes
    for name, L, K, n, seed in [("rq_syn_3x256", 3, 256, 8192, 1), ("rq_syn_4x1024", 4, 1024, 8192, 2)]:
        x, sha = gl.synth_items(n, mu, sigma, seed)
        sd, out, meta = make_rq(RQVAE, name, x, L, K, seed=seed)
        meta.update(x_seed=seed, x_sha256=sha)
        save(name, sd, out, meta, keep_z=(K == 256))
    # --- RQ-VAE: reference's own random codebook init (uniform +-1/K, vq.py:24): near-tie stress
    x, sha = gl.synth_items(2048, mu, sigma, 3)
    sd, out, meta = make_rq(RQVAE, "rq_syn_randinit_3x256", x, 3, 256, seed=3, data_codebooks=False)
    meta.update(x_seed=3, x_sha256=sha)
    save("rq_syn_randinit_3x256", sd, out, meta, keep_z=False)

    # --- SASRec config 1: CSV -> per-student sequences, SASRec/main.py params, untouched init
    users = {}
    for s, c in zip(students, class_ids):
        users.setdefault(s, []).append(int(c))
    n = 20
    seqs, targets = [], []
    for s, items in users.items():
        if len(items) < 3:   # min_seq_len (SASRec/main.py:35, data_vision.py:24)
            continue
        hist = items[:-1][-n:]
        seqs.append([0] * (n - len(hist)) + hist)
        targets.append(items[-1])
    seqs, targets = np.array(seqs, np.int64), np.array(targets, np.int64)
    item_num = int(class_ids.max())
    sd, out, meta = make_sasrec(SASRec, "sas_csv_c1", item_num, sas_params(16, 20, 2, 1, 64), seqs,
                                seed=0, perturb=False, targets=targets, n_forward=len(seqs))
    save("sas_csv_c1", sd, out, meta)
    # --- SASRec synthetic: C3 shape (small catalog), C5 shape, even heads (fast path)
    rng = np.random.default_rng(11)
    cases = [("sas_syn_c3", 2000, sas_params(64, 50, 2, 1, 64), 128),
             ("sas_syn_c5", 3000, sas_params(128, 200, 2, 1, 64), 48),
             ("sas_syn_h2", 1500, sas_params(64, 50, 2, 2, 64), 64),
             ("sas_syn_d32_h4", 999, sas_params(32, 37, 3, 4, 48), 40)]
    for i, (name, item_num, p, B) in enumerate(cases):
        seqs = random_seqs(rng, B, p["max_len"], item_num)
        sd, out, meta = make_sasrec(SASRec, name, item_num, p, seqs, seed=20 + i,
                                    n_forward=2 if p["max_len"] > 100 else 8)
        save(name, sd, out, meta)


if __name__ == "__main__":
    main()
