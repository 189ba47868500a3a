"""Calibration of the near-tie certificate's encoder bound ``Z_TAU`` on HELD-OUT fixtures.

``gr_amd.rqvae.Z_TAU`` bounds ``|z_gpu - z_ref| / |z_ref|`` per row (the fp32 encoder's deviation
from the reference's CPU/MKL bits).  It is set to 3x the largest ratio measured HERE, on
``rq_calib_3x256`` (16,384 rows, the C2/C4 encoder) and ``rq_calib_wide_3x256`` (4,096 rows, the
reference-default widths 768 -> [512, 256, 128] -> 64), whose weights and inputs are disjoint
from every fixture the certificate is then tested on (tests/golden/make_golden_calib.py).  The
out-of-sample check is ``test_encoder_latents_close_to_reference`` (rq_syn_3x256).
"""
import numpy as np
import pytest
import torch

import golden_lib as gl

pytestmark = pytest.mark.gpu
CALIB = ["rq_calib_3x256", "rq_calib_wide_3x256"]


@pytest.fixture(params=[1, 0], ids=["fused", "layerwise"])
def rq_path(request):
    from gr_amd import _lib
    _lib.set_option("rq_fused", request.param)
    yield request.param
    _lib.set_option("rq_fused", 1)


@pytest.mark.parametrize("name", CALIB)
def test_z_tau_has_3x_headroom_on_held_out(name, dev, rq_path, parity_log):
    from gr_amd import RQVAE, ops
    from gr_amd.rqvae import Z_TAU
    x, sd, out, meta = gl.rq_inputs(name)
    m = RQVAE(in_dim=768, num_emb_list=[meta["K"]] * meta["L"], e_dim=meta["e_dim"], layers=meta["layers"],
              sk_epsilons=[0.0] * meta["L"])
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    m = m.to(dev).eval()
    lin = m.encoder.linears()
    idx, z = ops.rq_encode(torch.from_numpy(x).to(dev), [l.weight for l in lin], [l.bias for l in lin],
                           m.rq.codebooks(), with_z=True)
    zr = out["z"].astype(np.float64)
    row = np.linalg.norm(z.cpu().numpy().astype(np.float64) - zr, axis=1) / np.linalg.norm(zr, axis=1)
    diff = (idx.cpu().numpy() != out["idx_full"]).any(1)
    parity_log(kind="z_tau_calibration", fixture=name, path="fused" if rq_path else "layerwise",
               rows=len(row), max_row_ratio=float(row.max()), p999_row_ratio=float(np.quantile(row, 0.999)),
               median_row_ratio=float(np.median(row)), z_tau=Z_TAU, headroom=float(Z_TAU / row.max()),
               rows_differ=int(diff.sum()))
    assert row.max() * 3 <= Z_TAU * 1.0001, (row.max(), Z_TAU)
