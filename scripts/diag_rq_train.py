"""Where the captured RQ-VAE training step's time goes (bench rq_train_step configuration): device
time per replay of ops.RqTrainGraph with Sinkhorn at every level (main.py) and with the plain argmin
(sk_epsilons 0), and of the quantizer op alone on the step's latents."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import RQVAE, ops, synth  # noqa: E402

dev = torch.device("cuda:0")


def ev_ms(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


for eps in (0.01, 0.0):
    torch.manual_seed(11)
    m = RQVAE(in_dim=768, num_emb_list=[8, 8, 8], e_dim=32, layers=[256, 128], dropout_prob=0.1,
              quant_loss_weight=0.1, beta=0.25, kmeans_init=False, sk_epsilons=[eps] * 3, sk_iters=50)
    for q in m.rq.vq_layers:
        q.embedding.weight.data.normal_(0.0, 0.3)
    m = m.to(dev).train()
    opt = torch.optim.AdamW(m.parameters(), lr=torch.tensor(1e-3, device=dev), weight_decay=1e-4, capturable=True)
    x = synth.items(64, 13, dev)
    step = ops.RqTrainGraph(m, opt, x.clone(), sync=False)
    print(f"sk_eps {eps}: captured step {ev_ms(step.replay) * 1e3:7.1f} us", flush=True)
    with torch.no_grad():
        z = m.encoder.mlp_layers(x).contiguous()
    cbs = [q.embedding.weight.detach() for q in m.rq.vq_layers]
    print(f"sk_eps {eps}: quantizer forward alone {ev_ms(lambda: ops.rq_quantize_train(z, cbs, 0.25, [eps] * 3, 50)) * 1e3:7.1f} us"
          f"   rq_quantize_sk alone {ev_ms(lambda: ops.rq_quantize_sk(z, cbs, [eps] * 3, 50)) * 1e3:7.1f} us", flush=True)
