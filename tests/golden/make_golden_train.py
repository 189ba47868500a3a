"""Golden fixtures for SASRec training-side scoring (SASRec/train.py:131-167).

Container-only (imports SASRec/model.py from /root/reference, read-only, never shipped):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_train.py

The reference model (train mode, dropout 0 so the forward is deterministic) produces
``seq_features`` for train-mode samples (data_vision.py:55-72: input = last n of seq[:-1], target =
last n of seq[1:], both left-padded with 0); negatives follow get_neg_samples (train.py:15-30) with a
seeded RandomState.  The loss block itself (train.py:134-167) is inline in the reference's train()
(its module imports h5py, absent here), so it runs from the oracle's verbatim restatement
(oracle/sasrec_oracle.train_loss).  Stored: features, item table, targets, negatives, batch loss,
valid count and the gradients of ``loss = batch_loss / valid`` w.r.t. features and table; the model's
state dict and the gradient of every parameter for the whole step (forward under autograd, loss,
backward through the reference model).
"""
import json
import os
import sys

sys.dont_write_bytecode = True
import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import sasrec_oracle  # noqa: E402

REF = "/root/reference"
torch.set_num_threads(8)


def _ref_sasrec():
    sys.path.insert(0, os.path.join(REF, "SASRec"))
    import model as m  # noqa
    sys.path.pop(0)
    return m.SASRec


def train_samples(rng, B, n, item_num, edge=True):
    seqs, tgts = np.zeros((B, n), np.int64), np.zeros((B, n), np.int64)
    for b in range(B):
        L = int(rng.integers(3, n + 8))
        seq = rng.permutation(np.arange(1, item_num + 1))[:L]      # distinct items, like real histories
        if edge and b == 1:
            seq = seq[:2]                                            # shortest history: one position
        inp, tgt = seq[:-1][-n:], seq[1:][-n:]
        seqs[b, n - len(inp):] = inp
        tgts[b, n - len(tgt):] = tgt
    return seqs, tgts


def make(SASRec, name, item_num, d, n, B, J, seed, mlp=64, heads=1, blocks=2, eps=1e-24):
    torch.manual_seed(seed)
    params = {"device": "cpu", "d": d, "max_len": n, "num_blocks": blocks, "num_heads": heads,
              "dropout": 0.0, "mlp_layer": mlp, "layernorm_eps": 1e-8}
    model = SASRec(item_num, params).train()
    rng = np.random.default_rng(seed)
    seqs, tgts = train_samples(rng, B, n, item_num)
    negs = sasrec_oracle.neg_samples(seqs, item_num, J, np.random.RandomState(seed))
    tg = torch.from_numpy(tgts)
    # edge: one negative equal to the user's last target (allowed: get_neg_samples only excludes the
    # input history, and the last target is not in it), so one score is gathered twice
    negs[0, 0] = tg[0, -1]
    with torch.no_grad():
        feats = model(torch.from_numpy(seqs)).detach()
    table = model.item_emb.weight.detach().clone()
    bl, valid, gf, gw = sasrec_oracle.train_loss_grads(feats, table, tg, negs, eps)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    # the whole train.py:131-167 step through the reference model: forward (autograd), loss, backward
    model.zero_grad()
    f2 = model.forward(torch.from_numpy(seqs))
    bl2, valid2 = sasrec_oracle.train_loss(f2, model.item_emb.weight, tg, negs, eps)
    (bl2 / valid2.item()).backward()
    pgrads = {f"pgrad/{k}": p.grad.detach().numpy() for k, p in model.named_parameters() if p.grad is not None}
    meta = dict(name=name, item_num=item_num, d=d, n=n, B=B, num_neg=J, eps=eps, seed=seed,
                params=params, torch=torch.__version__)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), meta=json.dumps(meta),
                        feats=feats.numpy(), table=table.numpy(), targets=tgts, negs=negs.numpy(),
                        seqs=seqs, batch_loss=np.float32(bl.item()), valid=np.float32(valid.item()),
                        dfeats=gf.numpy(), dtable=gw.numpy(), **{f"sd/{k}": v.numpy() for k, v in sd.items()},
                        **pgrads)
    print(name, "batch_loss", bl.item(), "valid", valid.item())


def main():
    SASRec = _ref_sasrec()
    make(SASRec, "sas_train_main", 300, 16, 20, 32, 10, 11)          # SASRec/main.py:6-42 shapes
    make(SASRec, "sas_train_d64", 2000, 64, 50, 16, 10, 12)          # C3 shapes (d 64, n 50)
    make(SASRec, "sas_train_d128", 1000, 128, 30, 8, 5, 13, heads=2)


if __name__ == "__main__":
    main()
