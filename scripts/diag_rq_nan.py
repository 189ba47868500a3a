"""Diagnostic: the eager RQ-VAE train step of tests/test_rq_train_gpu.py (dropout 0, foreach
capturable AdamW), checking every stage for non-finite values."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_rq_train_gpu import _model, _opt, _batches  # noqa: E402

dev = torch.device("cuda:0")
for trial in range(1):
    for fused, kern in ((None, True), (False, True), (False, False), (True, True)):
        m = _model(dev, 0.0, False)
        m.encoder.fused_train = m.decoder.fused_train = m.rq.fused_train = kern
        opt, sch = _opt(m, dev, warm=1, fused=fused)
        for it, x in enumerate(_batches(dev, 4)):
            opt.zero_grad(set_to_none=True)
            o, rq_loss, idx = m(x)
            loss, recon = m.compute_loss(o, rq_loss, xs=x)
            bad = {"out": not torch.isfinite(o).all().item(), "rq_loss": not torch.isfinite(rq_loss).item()}
            loss.backward()
            for k, p in m.named_parameters():
                if p.grad is None or not torch.isfinite(p.grad).all():
                    bad["grad " + k] = True
            torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            opt.step()
            sch.step()
            for k, p in m.named_parameters():
                if not torch.isfinite(p).all():
                    bad["param " + k] = True
            bad = [k for k, v in bad.items() if v]
            print(f"kernels {kern} fused {fused} step {it}: loss {loss.item():.5f} lr {opt.param_groups[0]['lr'].item():.2e} bad {bad}", flush=True)
