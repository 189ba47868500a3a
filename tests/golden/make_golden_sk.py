"""Golden fixtures for RQVAE.get_indices(use_sk=True) and the RQ-VAE/infer.py code-emission tail
(collision rounds + dedup digit), produced by running the REFERENCE model on CPU in the build
container (container-only; imports RQ-VAE/models from /root/reference, writes only .npz data).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_sk.py
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
from oracle import rq_oracle  # noqa: E402

REF = "/root/reference"
torch.set_num_threads(8)


def ref_model(L, K, sd, sk_eps, sk_iters=50):
    sys.path.insert(0, os.path.join(REF, "RQ-VAE"))
    from models.rqvae import RQVAE  # noqa
    sys.path.pop(0)
    m = RQVAE(in_dim=768, num_emb_list=[K] * L, e_dim=32, layers=[256, 128], dropout_prob=0.1, bn=False,
              loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=False, kmeans_iters=50,
              sk_epsilons=list(sk_eps), sk_iters=sk_iters).eval()
    m.load_state_dict({k: torch.as_tensor(v) for k, v in sd.items()}, strict=False)
    return m


@torch.no_grad()
def ref_infer(model, x, batch_size=64, max_rounds=30):
    """The model-facing part of RQ-VAE/infer.py:88-162, driven through the reference model."""
    xt = torch.from_numpy(x)
    codes = torch.cat([model.get_indices(xt[i:i + batch_size], use_sk=False)
                       for i in range(0, len(xt), batch_size)]).numpy()
    initial = codes.copy()
    for vq in model.rq.vq_layers[:-1]:          # infer.py:109-110
        vq.sk_epsilon = 0.0
    rounds, outs = [], []
    for _ in range(max_rounds):
        groups = rq_oracle.collision_groups(codes)
        if not groups:
            break
        rounds.append(groups)
        for g in groups:
            o = model.get_indices(xt[g], use_sk=True).numpy()
            outs.append(o)
            codes[g] = o
    return initial, codes, rq_oracle.dedup_codes(codes), rounds, outs


def flat(groups_per_round):
    rows, ptr, rnd = [], [0], []
    for r, groups in enumerate(groups_per_round):
        for g in groups:
            rows.extend(g)
            ptr.append(len(rows))
            rnd.append(r)
    return np.array(rows, np.int64), np.array(ptr, np.int64), np.array(rnd, np.int64)


def make_case(name, x, sd, L, K, meta_extra):
    model = ref_model(L, K, sd, [0.01] * L)
    initial, codes, final, rounds, outs = ref_infer(model, x)
    ws, bs, cbs = rq_oracle.state_to_lists({k: torch.as_tensor(v) for k, v in sd.items()}, L)
    o_codes, o_final, o_rounds = rq_oracle.infer_codes(torch.from_numpy(x), ws, bs, cbs, [0.01] * L, 50)
    assert np.array_equal(o_final, final) and o_rounds == rounds, f"{name}: oracle != reference"
    rows, ptr, rnd = flat(rounds)
    # direct get_indices(use_sk=True) with Sinkhorn at EVERY level on the first-round groups
    model_all = ref_model(L, K, sd, [0.01] * L)
    g0 = rounds[0] if rounds else []
    xt = torch.from_numpy(x)
    direct = [model_all.get_indices(xt[g], use_sk=True).numpy() for g in g0]
    r0, p0, _ = flat([g0])
    o_direct = [rq_oracle.get_indices_sk(xt[g], ws, bs, cbs, [0.01] * L, 50).numpy() for g in g0]
    assert all(np.array_equal(a, b) for a, b in zip(direct, o_direct)), f"{name}: sk oracle != reference"
    out = dict(initial=initial, codes=codes, final=final, round_rows=rows, round_ptr=ptr, round_id=rnd,
               round_out=np.concatenate(outs) if outs else np.zeros((0, L), np.int64),
               all_rows=r0, all_ptr=p0,
               all_out=np.concatenate(direct) if direct else np.zeros((0, L), np.int64))
    meta = dict(name=name, L=L, K=K, n=len(x), sk_eps=0.01, sk_iters=50, rounds=len(rounds),
                groups=int(len(ptr) - 1), torch=torch.__version__, **meta_extra)
    arrs = {f"sd/{k}": np.asarray(v) for k, v in sd.items() if not k.startswith("decoder.")}
    arrs.update(out)
    arrs["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(name, meta, "final unique:", len(np.unique(final, axis=0)), "/", len(final))


def main():
    # config-1 data (80 real BERT vectors), the 3x8 model of rq_csv_3x8
    x, sd, _, meta = gl.rq_inputs("rq_csv_3x8")
    make_case("rq_sk_csv_3x8", x, sd, 3, 8, {"src": "rq_csv_3x8"})
    # synthetic 2048 items, 3x16 data-derived codebooks: many collision groups
    c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
    xs, sha = gl.synth_items(2048, c["mu"], c["sigma"], 11)
    sys.path.insert(0, os.path.join(REF, "RQ-VAE"))
    from models.rqvae import RQVAE  # noqa
    sys.path.pop(0)
    torch.manual_seed(11)
    m = RQVAE(in_dim=768, num_emb_list=[16] * 3, e_dim=32, layers=[256, 128], dropout_prob=0.1,
              sk_epsilons=[0.01] * 3, sk_iters=50).eval()
    with torch.no_grad():
        r = m.encoder(torch.from_numpy(xs))
        for l, vq in enumerate(m.rq.vq_layers):
            g = torch.Generator().manual_seed(50 + l)
            pick = torch.randperm(r.shape[0], generator=g)[:16]
            vq.embedding.weight.copy_(r[pick] + 0.01 * r.std() * torch.randn((16, r.shape[1]), generator=g))
            x_res, _, _ = vq(r, use_sk=False)
            r = r - x_res
    sd2 = {k: v.detach().clone().numpy() for k, v in m.state_dict().items()}
    make_case("rq_sk_syn_3x16", xs, sd2, 3, 16, {"x_seed": 11, "x_sha256": sha})


if __name__ == "__main__":
    main()
