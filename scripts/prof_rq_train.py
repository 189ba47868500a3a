"""Replays of the captured RQ-VAE training step only (bench rq_train_step configuration), for
rocprofv3 --kernel-trace: what one replay launches and how long each kernel runs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import RQVAE, ops, synth  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(11)
m = RQVAE(in_dim=768, num_emb_list=[8, 8, 8], e_dim=32, layers=[256, 128], dropout_prob=0.1,
          quant_loss_weight=0.1, beta=0.25, kmeans_init=False, sk_epsilons=[0.01] * 3, sk_iters=50)
for q in m.rq.vq_layers:
    q.embedding.weight.data.normal_(0.0, 0.3)
m = m.to(dev).train()
opt = torch.optim.AdamW(m.parameters(), lr=torch.tensor(1e-3, device=dev), weight_decay=1e-4, capturable=True,
                        fused=True)
step = ops.RqTrainGraph(m, opt, synth.items(64, 13, dev), sync=False)
torch.cuda.synchronize()
for _ in range(int(os.environ.get("GR_REPLAYS", "20"))):
    step.replay()
torch.cuda.synchronize()
