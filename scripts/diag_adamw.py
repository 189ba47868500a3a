"""Diagnostic: torch AdamW(capturable=True, tensor lr) foreach vs fused on this ROCm build, on a plain
parameter with a plain gradient (no gr_amd kernels)."""
import torch

dev = torch.device("cuda:0")
for fused in (None, False, True):
    for wd in (0.0, 1e-4):
        p = torch.nn.Parameter(torch.randn(256, 768, device=dev))
        opt = torch.optim.AdamW([p], lr=torch.tensor(1e-3, device=dev), weight_decay=wd, capturable=True, fused=fused)
        p.grad = torch.randn_like(p) * 1e-2
        opt.step()
        print(f"fused={fused} wd={wd}: finite {torch.isfinite(p).all().item()}  "
              f"defaults fused={opt.defaults.get('fused')} foreach={opt.defaults.get('foreach')}", flush=True)
