"""Diagnostic: gradients of one captured training step (ops.SasTrainGraph, fused training kernels)
vs the same step issued eagerly, SGD with lr 0 so the parameters stay put."""
import copy
import sys

import torch

sys.path.insert(0, "/root/repo")
from gr_amd import ops, synth  # noqa: E402

dev = torch.device("cuda:0")
B, n, d, items, J = 32, 20, 64, 3000, 5
p = synth.sasrec_params(d, n, 2, 1, 64, dev)
p["dropout"] = 0.0
m = synth.sasrec_model(items, p, dev, seed=7).train()
ref = copy.deepcopy(m)
opt = torch.optim.SGD(m.parameters(), lr=0.0)
g = torch.Generator(device=dev).manual_seed(9)
seqs = torch.randint(1, items + 1, (B, n), generator=g, device=dev)
seqs[:, :3] = 0
targets = torch.roll(seqs, -1, dims=1)
targets[:, -1] = torch.randint(1, items + 1, (B,), generator=g, device=dev)
targets[seqs == 0] = 0
lr = float(sys.argv[2]) if len(sys.argv) > 2 else 0.05
for x in opt.param_groups:
    x["lr"] = lr
ref_opt = torch.optim.SGD(ref.parameters(), lr=lr)
step = ops.SasTrainGraph(m, opt, seqs, targets, items, J, 1e-24, seed=21)
for it in range(3):
    key = int(step.seed.item())
    bl, valid = step.replay()
    negs = ops.neg_samples(seqs, items, J, seed_tensor=torch.tensor([key], dtype=torch.int64, device=dev))
    ref_opt.zero_grad()
    bl2, valid2 = ops.sampled_bce_loss(ref(seqs), ref.item_emb.weight, targets, negs, 1e-24)
    (bl2 / valid2).backward()
    gdiff = {name: float((a.grad - b.grad).abs().max()) for (name, a), b in zip(m.named_parameters(), ref.parameters())
             if a.grad is not None and b.grad is not None}
    ref_opt.step()
    pdiff = max(float((a - b).abs().max()) for a, b in zip(m.parameters(), ref.parameters()))
    worst = sorted(gdiff.items(), key=lambda kv: -kv[1])[:3]
    ig = m.item_emb.weight.grad
    print(f"  graph item grad max {float(ig.abs().max()):.3e} eager {float(ref.item_emb.weight.grad.abs().max()):.3e}; "
          f"rows with |diff|>1e-3: {int(((ig - ref.item_emb.weight.grad).abs().amax(1) > 1e-3).sum())}; grad ptr {ig.data_ptr():#x}", flush=True)
    print(f"step {it}: loss graph {float(bl):.4f} eager {float(bl2.detach()):.4f}; max param diff after step {pdiff:.3e}; worst grad diffs {worst}", flush=True)
