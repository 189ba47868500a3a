"""Held-out fixtures for calibrating the near-tie certificate's encoder bound ``Z_TAU``.

Container-only (imports the reference's ``RQ-VAE/models`` like make_golden.py).  The fixtures
written here are used for ONE thing: measuring how far the GPU encoder's fp32 output may sit from
the reference's CPU/MKL output (per row, ``|dz| / |z|``).  ``gr_amd.rqvae.Z_TAU`` is set from that
measurement (tests/test_rq_calib_gpu.py, profiles/r02_ztau_calibration.json), and the certificate
is then exercised on the OTHER fixtures (rq_csv_3x8, rq_syn_*), which never fed the calibration.

Seeds, encoder weights and inputs are disjoint from make_golden.py's (x seeds 101/102, model seeds
41/42), and two encoder shapes are covered: the C2/C4 encoder 768 -> [256, 128] -> 32 and the
reference's default-width 768 -> [512, 256, 128] -> 64 (RQ-VAE/models/rqvae.py:10-27).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_calib.py
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

CASES = [  # name, n, L, K, e_dim, layers, x seed, model seed
    ("rq_calib_3x256", 16384, 3, 256, 32, (256, 128), 101, 41),
    ("rq_calib_wide_3x256", 4096, 3, 256, 64, (512, 256, 128), 102, 42),
]


def main():
    RQVAE, _ = mg._import_ref()
    c = np.load(os.path.join(HERE, "csv_bert.npz"), allow_pickle=False)
    for name, n, L, K, e, layers, xs, ms in CASES:
        x, sha = gl.synth_items(n, c["mu"], c["sigma"], xs)
        sd, out, meta = mg.make_rq(RQVAE, name, x, L, K, seed=ms, e_dim=e, layers=layers)
        meta.update(x_seed=xs, x_sha256=sha, purpose="Z_TAU calibration only (held out)")
        arrs = {f"sd/{k}": v.numpy() for k, v in sd.items() if not k.startswith("decoder.")}
        arrs.update({k: v for k, v in out.items() if k in ("z", "idx_full", "gap", "dbest", "znorm")})
        arrs["meta"] = np.array(json.dumps(meta))
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
        print(name, {k: v for k, v in meta.items() if k != "x_sha256"})


if __name__ == "__main__":
    main()
