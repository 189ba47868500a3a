"""Golden fixture for a BatchNorm encoder: ``RQVAE(bn=True)`` (RQ-VAE/models/layers.py:25-26) in
eval mode, with non-trivial running statistics and affine parameters.

Container-only (imports the reference's ``RQ-VAE/models`` like make_golden.py); writes
tests/golden/rq_bn_3x256.npz (state dict incl. the BatchNorm buffers, inputs by seed, the
reference's get_indices, encoder output and the near-tie certificate inputs).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_bn.py
"""
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import golden_lib as gl  # noqa: E402
import make_golden as mg  # noqa: E402
from oracle import rq_oracle  # noqa: E402


def main():
    RQVAE, _ = mg._import_ref()
    c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
    name, n, L, K, seed, xs = "rq_bn_3x256", 4096, 3, 256, 51, 103
    x, sha = gl.synth_items(n, c["mu"], c["sigma"], xs)
    xt = torch.from_numpy(x)
    torch.manual_seed(seed)
    model = RQVAE(in_dim=768, num_emb_list=[K] * L, e_dim=32, layers=[256, 128], dropout_prob=0.1, bn=True,
                  loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=False, kmeans_iters=50,
                  sk_epsilons=[0.0] * L, sk_iters=50)
    g = torch.Generator().manual_seed(seed + 1)
    with torch.no_grad():
        # running statistics as a few training batches would leave them (train-mode passes), then
        # perturbed affine parameters
        model.train()
        for i in range(4):
            model.encoder(xt[i * 512:(i + 1) * 512])
        for m in model.encoder.mlp_layers:
            if isinstance(m, torch.nn.BatchNorm1d):
                m.weight.copy_(1.0 + 0.1 * torch.randn(m.weight.shape, generator=g))
                m.bias.copy_(0.05 * torch.randn(m.bias.shape, generator=g))
        model.eval()
        z = model.encoder(xt)
        r = z
        for l, vq in enumerate(model.rq.vq_layers):   # data-derived codebooks (make_golden.make_rq)
            gg = torch.Generator().manual_seed(seed + 10 + l)
            pick = torch.randperm(n, generator=gg)[:K]
            vq.embedding.weight.copy_(r[pick] + 0.01 * r.std() * torch.randn((K, r.shape[1]), generator=gg))
            x_res, _, _ = vq(r, use_sk=False)
            r = r - x_res
        idx = model.get_indices(xt, use_sk=False)
        cbs = [q.embedding.weight.detach().clone() for q in model.rq.vq_layers]
        ref, residuals, gaps = rq_oracle.rq_quantize(z, cbs, return_detail=True)
        assert torch.equal(ref, idx)
        dbest = torch.stack([rq_oracle.vq_level(rr, cb)[2].min(1).values for rr, cb in zip(residuals, cbs)], -1)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items() if not k.startswith("decoder.")}
    meta = dict(name=name, L=L, K=K, e_dim=32, layers=[256, 128], in_dim=768, n=n, seed=seed, bn=True,
                x_seed=xs, x_sha256=sha, torch=torch.__version__, data_codebooks=True)
    arrs = {f"sd/{k}": v.numpy() for k, v in sd.items()}
    arrs.update(idx_full=idx.numpy(), z=z.numpy(), gap=gaps.numpy(), dbest=dbest.numpy(),
                znorm=(z ** 2).sum(1).numpy())
    arrs["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(name, {k: v for k, v in meta.items() if k != "x_sha256"})


if __name__ == "__main__":
    main()
