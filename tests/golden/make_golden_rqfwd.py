"""Golden fixtures for the RQ-VAE training forward (rqvae.py:60-65 + compute_loss :73-84; SURVEY §8(f)
row 4: "RQ-VAE forward with Sinkhorn every step", the RQ-VAE/train.py:113-116 call).

Container-only (imports RQ-VAE/models from /root/reference, read-only, never shipped):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_rqfwd.py

Runs the reference RQVAE itself: ``out, rq_loss, indices = model(x, use_sk)`` and
``loss, recon = model.compute_loss(out, rq_loss, xs=x)``, then ``loss.backward()``, in eval mode
(dropout off; k-means init off — sklearn's KMeans is randomly seeded — with data-derived codebooks
instead).  Stored: inputs, state dict, out, rq_loss, indices, loss, recon and every parameter's grad.
"""
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import golden_lib as gl  # noqa: E402

REF = "/root/reference"
torch.set_num_threads(8)


def _ref_rqvae():
    sys.path.insert(0, os.path.join(REF, "RQ-VAE"))
    from models.rqvae import RQVAE  # noqa
    sys.path.pop(0)
    return RQVAE


def make(RQVAE, name, x, K, L, sk_eps, use_sk, seed, sk_iters=50):
    torch.manual_seed(seed)
    model = RQVAE(in_dim=768, num_emb_list=[K] * L, e_dim=32, layers=[256, 128], dropout_prob=0.1,
                  bn=False, loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=False,
                  kmeans_iters=50, sk_epsilons=sk_eps, sk_iters=sk_iters).eval()
    xt = torch.from_numpy(x)
    with torch.no_grad():
        r = model.encoder(xt)
        for l, vq in enumerate(model.rq.vq_layers):   # data-derived codebooks (k-means-like init)
            g = torch.Generator().manual_seed(seed + 1 + l)
            pick = torch.randperm(r.shape[0], generator=g)[:K]
            vq.embedding.weight.copy_(r[pick] + 0.05 * r.std() * torch.randn((K, r.shape[1]), generator=g))
            x_res, _, _ = vq(r, use_sk=False)
            r = r - x_res
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    with torch.no_grad():
        out_ng, loss_ng, idx_ng = model(xt, use_sk=use_sk)
    model.zero_grad()
    out, rq_loss, idx = model(xt, use_sk=use_sk)
    loss, recon = model.compute_loss(out, rq_loss, xs=xt)
    loss.backward()
    assert torch.equal(idx, idx_ng) and torch.equal(out, out_ng)
    grads = {f"grad/{k}": p.grad.detach().numpy() for k, p in model.named_parameters() if p.grad is not None}
    meta = dict(name=name, K=K, L=L, sk_eps=sk_eps, sk_iters=sk_iters, use_sk=use_sk, seed=seed, n=len(x),
                torch=torch.__version__)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), meta=json.dumps(meta), x=x,
                        **{f"sd/{k}": v.numpy() for k, v in sd.items()},
                        out=out.detach().numpy(), rq_loss=np.float32(rq_loss.item()), indices=idx.numpy(),
                        loss=np.float32(loss.item()), recon=np.float32(recon.item()), **grads)
    print(name, "loss", loss.item(), "rq_loss", rq_loss.item(), "distinct codes",
          len({tuple(r) for r in idx.tolist()}))


def main():
    RQVAE = _ref_rqvae()
    c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
    # RQ-VAE/main.py: [8, 8, 8], sk_epsilons 0.01 at every level, batch 64 (the 80 CSV vectors' first 64)
    make(RQVAE, "rqfwd_main_sk", c["vecs"][:64].astype(np.float32), 8, 3, [0.01] * 3, True, 21)
    x, _ = gl.synth_items(512, c["mu"], c["sigma"], 22)
    make(RQVAE, "rqfwd_3x256_nosk", x, 256, 3, [0.0] * 3, False, 23)
    make(RQVAE, "rqfwd_3x64_sk_last", x[:256], 64, 3, [0.0, 0.0, 0.003], True, 24)


if __name__ == "__main__":
    main()
