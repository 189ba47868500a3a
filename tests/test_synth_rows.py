"""synth.table_rows / sasrec_rank_model: the position-keyed synthetic item table the C5 bench builds
per rank (each rank builds only its catalog shard), so every world size scores
the same table and the cross-rank result checksum is comparable between N = 1 and N = 8."""
import numpy as np
import pytest
import torch

from gr_amd import dist as D, synth


def test_table_rows_are_position_keyed():
    full = synth.table_rows(torch.arange(0, 5000), 128, 7, "cpu")
    assert full.dtype == torch.float32 and full.shape == (5000, 128)
    assert torch.count_nonzero(full[0]) == 0                      # padding_idx = 0
    for world in (2, 3, 8):
        parts = [synth.table_rows(torch.arange(*D.shard_range(5000, r, world)), 128, 7, "cpu") for r in range(world)]
        assert torch.equal(torch.cat(parts), full)
    ids = torch.tensor([4999, 17, 0, 17, 1234])
    assert torch.equal(synth.table_rows(ids, 128, 7, "cpu"), full[ids])
    other = synth.table_rows(torch.arange(1, 5000), 128, 8, "cpu")
    assert not torch.equal(other, full[1:])                       # the seed matters
    x = full[1:].double()
    assert abs(float(x.mean())) < 0.01 and abs(float(x.std()) - 1.0) < 0.01
    assert bool(torch.isfinite(full).all())


def test_rank_model_compact_table():
    p = synth.sasrec_params(32, 20, 2, 1, 64, "cpu")
    seqs = synth.sequences(6, 20, 1000, 1, "cpu")
    m, cs = synth.sasrec_rank_model(1000, p, seqs, "cpu", seed=5)
    used = torch.unique(torch.cat([torch.zeros(1, dtype=seqs.dtype), seqs.reshape(-1)]))
    assert m.item_emb.weight.shape == (used.numel(), 32) and m.item_num == used.numel() - 1
    assert torch.equal(used[cs], seqs)                             # the remap is exact
    assert torch.equal(m.item_emb.weight[cs], synth.table_rows(seqs.reshape(-1), 32, 7, "cpu").view(6, 20, 32))
    # the transformer parameters do not depend on which rows a rank holds
    m2, _ = synth.sasrec_rank_model(1000, p, seqs[3:], "cpu", seed=5)
    for (k, v), (k2, v2) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2
        if k != "item_emb.weight":
            assert torch.equal(v, v2), k
    with pytest.raises(IndexError):
        synth.sasrec_rank_model(10, p, seqs, "cpu")
