"""Helpers shared by the fixture generator and the tests (no reference code, no reference import)."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def synth_items(n, mu, sigma, seed):
    """Synthetic BERT-like item embeddings ``x = mu + sigma * eps``.

    ``eps`` comes from numpy's PCG64 generator in float32, so the bytes are reproducible on any
    host with the same numpy; the SHA-256 of the bytes is returned for verification.
    """
    eps = np.random.default_rng(seed).standard_normal((n, mu.shape[0]), dtype=np.float32)
    x = (mu.astype(np.float32)[None, :] + sigma.astype(np.float32)[None, :] * eps).astype(np.float32)
    return x, hashlib.sha256(x.tobytes()).hexdigest()


def load(name):
    """Load ``tests/golden/<name>.npz`` -> (state_dict as numpy, outputs, meta)."""
    z = np.load(os.path.join(HERE, f"{name}.npz"), allow_pickle=False)
    sd = {k[3:]: z[k] for k in z.files if k.startswith("sd/")}
    out = {k: z[k] for k in z.files if not k.startswith("sd/") and k != "meta"}
    meta = json.loads(str(z["meta"]))
    return sd, out, meta


def rq_inputs(name):
    """The item embeddings a RQ fixture was generated from (CSV vectors or regenerated synthetic)."""
    sd, out, meta = load(name)
    if meta["name"].startswith("rq_csv"):
        x = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)["vecs"]
    else:
        c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
        x, sha = synth_items(meta["n"], c["mu"], c["sigma"], meta["x_seed"])
        assert sha == meta["x_sha256"], "synthetic input regeneration is not bit-exact on this host"
    return x, sd, out, meta
