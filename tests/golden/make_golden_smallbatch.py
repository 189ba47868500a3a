"""Golden fixtures for the reference's SMALL get_indices calls (container-only; imports the
reference from /root/reference, emits only data).

MKL's CPU sgemm takes other accumulation orders for calls of 1-15 rows (oracle/rq_exact.c rqx_plan),
so the reference's semantic IDs depend on the call's batch size there.  Two call patterns of the
reference hit it:
  * the tail batch of its DataLoader(bs=64) loop (RQ-VAE/infer.py:84-95, generate_code.py:78-88)
    when n mod 64 is 1..15 -- e.g. the real 707-item catalog (RQVAE-T5/data_read.ipynb: (707, 4));
  * the collision re-encode of tiny groups (infer.py:121-122; Sinkhorn, covered by rq_sk_*).
This writes, for the rq_csv_3x8 / rq_syn_3x256 / rq_syn_4x1024 models and rq_syn_randinit_3x256
(the reference's own uniform(+-1/K) codebook init: near-tie heavy, so the small-call encoder bits
move IDs there):
  small_M{m}  get_indices on 24 (randinit: 192) windows of m consecutive rows, m = 1..17
              ([windows, m, L]; starts in small_starts_M{m}), z_M{m} the encoder outputs of the same
              calls (rq_syn_3x256);
  b64_707     the batch-64 loop over a 707-item synthetic catalog (a 3-row tail) and b64_707_full
              the same items in one call.
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_smallbatch.py
"""
import json
import os
import platform
import sys

sys.dont_write_bytecode = True
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import golden_lib as gl  # noqa: E402
from oracle import rq_exact  # noqa: E402

REF = "/root/reference"
torch.set_num_threads(8)
WINDOWS = 24


def host_meta():
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), "")
    except OSError:
        pass
    mkl = [l.strip() for l in torch.__config__.show().splitlines() if "Math Kernel" in l]
    return dict(cpu=cpu, machine=platform.machine(), torch=torch.__version__, threads=torch.get_num_threads(),
                mkl=mkl[0] if mkl else "", capability=torch.backends.cpu.get_cpu_capability())


def ref_model(RQVAE, sd, meta):
    L, K = meta["L"], meta["K"]
    m = RQVAE(in_dim=meta["in_dim"], num_emb_list=[K] * L, e_dim=meta["e_dim"], layers=list(meta["layers"]),
              dropout_prob=0.1, bn=False, loss_type="mse", quant_loss_weight=0.1, beta=0.25, kmeans_init=False,
              kmeans_iters=50, sk_epsilons=[0.01] * L, sk_iters=50).eval()
    own = m.state_dict()
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items() if k in own}, strict=False)
    return m


def main():
    sys.path.insert(0, os.path.join(REF, "RQ-VAE"))
    from models.rqvae import RQVAE  # noqa
    sys.path.pop(0)
    c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
    cat, cat_sha = gl.synth_items(707, c["mu"], c["sigma"], 11)
    for name in ("rq_csv_3x8", "rq_syn_3x256", "rq_syn_4x1024", "rq_syn_randinit_3x256"):
        x, sd, _, meta = gl.rq_inputs(name)
        model = ref_model(RQVAE, sd, meta)
        xt = torch.from_numpy(x)
        ws = [sd[f"encoder.mlp_layers.{i}.weight"] for i in (1, 4, 7)]
        bs = [sd[f"encoder.mlp_layers.{i}.bias"] for i in (1, 4, 7)]
        cbs = [sd[f"rq.vq_layers.{l}.embedding.weight"] for l in range(meta["L"])]
        rng = np.random.default_rng(1234)
        nwin = WINDOWS * 8 if name == "rq_syn_randinit_3x256" else WINDOWS
        out = {}
        differ = {}
        with torch.no_grad():
            for m in range(1, 18):
                starts = rng.integers(0, x.shape[0] - m, nwin)
                idx = np.stack([model.get_indices(xt[s:s + m], use_sk=False).numpy() for s in starts])
                z = np.stack([model.encoder(xt[s:s + m]).numpy() for s in starts])
                out[f"small_M{m}"] = idx
                out[f"small_starts_M{m}"] = starts.astype(np.int64)
                if name == "rq_syn_3x256":
                    out[f"z_M{m}"] = z
                # the restatement must agree before anything is written
                for wi, s in enumerate(starts):
                    o_idx, o_z, _, _ = rq_exact.encode(x[s:s + m], ws, bs, cbs, with_detail=True)
                    assert np.array_equal(o_z, z[wi]), f"{name} M={m}: rq_exact z != reference"
                    assert np.array_equal(o_idx, idx[wi]), f"{name} M={m}: rq_exact idx != reference"
                # how often the small-call bits change the IDs against one long call
                full = rq_exact.encode(x[np.concatenate([np.arange(s, s + m) for s in starts])], ws, bs, cbs)
                differ[m] = int((full.reshape(idx.shape) != idx).any(-1).sum())
            ct = torch.from_numpy(cat)
            b64 = torch.cat([model.get_indices(ct[i:i + 64], use_sk=False) for i in range(0, 707, 64)]).numpy()
            full = model.get_indices(ct, use_sk=False).numpy()
        assert np.array_equal(rq_exact.encode_batches(cat, ws, bs, cbs, 64), b64), f"{name}: b64 loop"
        out["b64_707"] = b64
        out["b64_707_full"] = full
        m2 = dict(name=name, model_meta=meta, windows=nwin, cat_seed=11, cat_sha256=cat_sha, host=host_meta(),
                  windows_differing_from_long_call=differ,
                  b64_vs_full_rows=int((b64 != full).any(1).sum()))
        out["meta"] = np.array(json.dumps(m2))
        np.savez_compressed(os.path.join(HERE, f"{name}_small.npz"), **out)
        print(name, {k: v for k, v in m2.items() if k != "model_meta"})


if __name__ == "__main__":
    main()
