"""Fused rank (no logits) and the evaluation harness on the GPU.

Bar: target logits bitwise equal to the scoring kernel's entries; counts / ranks exactly equal to
the reference tail (evaluate.py:27-32) run on the GPU's own logits; ranks / HR@10 / NDCG@10 equal
to the golden fixtures."""
import os

import numpy as np
import pytest
import torch

import golden_lib as gl

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,d,rows", [(300, 64, 10001), (64, 128, 5000), (257, 32, 1000), (1, 64, 70),
                                      (70, 64, 64)])
def test_pairs_and_count_equal_materialised_logits(B, d, rows, dev):
    from gr_amd import ops
    g = torch.Generator().manual_seed(B * d + rows)
    h = torch.randn(B, d, generator=g).to(dev)
    t = torch.randn(rows, d, generator=g).to(dev)
    tg = torch.randint(0, rows, (B,), generator=g).to(dev)
    tg[0] = 0
    logits = ops.score(h, t)
    pairs = ops.score_pairs(h, t, tg, mask_col0=False)
    assert torch.equal(pairs, logits.gather(1, tg[:, None])[:, 0])   # bitwise the same chain
    lg = logits.clone()
    lg[:, 0] = -1e9
    ref = (lg > lg.gather(1, tg[:, None])).sum(1) + 1
    assert torch.equal(ops.score_rank(h, t, tg), ref)
    thr = torch.randn(B, generator=g).to(dev)
    assert torch.equal(ops.score_count_gt(h, t, thr, mask_col0=False), (logits > thr[:, None]).sum(1))


@pytest.mark.parametrize("d,n,items,B,heads", [(16, 20, 706, 128, 1), (16, 20, 706, 1, 1), (64, 50, 100_000, 128, 1),
                                                (32, 30, 5000, 300, 2), (128, 200, 20000, 64, 1), (64, 50, 3000, 2049, 1)])
def test_sasrec_rank_one_call_equals_materialised(d, n, items, B, heads, dev):
    """gr_sasrec_rank_f32 (forward + target logit + strict count + 1 in one call)
    against evaluate.py:27-32 run on the GPU's own predict() logits: equal ranks, every user; also
    with column 0 unmasked, and the one-call path through evaluate.rank_batch."""
    from gr_amd import ops, synth
    from gr_amd.evaluate import rank_batch
    p = synth.sasrec_params(d, n, 2, heads, 64, dev)
    m = synth.sasrec_model(items, p, dev, seed=d + n)
    seqs = synth.sequences(B, n, items, 31 + B, dev)
    g = torch.Generator(device=dev).manual_seed(B)
    tg = torch.randint(0, items + 1, (B,), generator=g, device=dev)
    tg[0] = 0
    logits = m.predict(seqs)
    lg = logits.clone()
    lg[:, 0] = -1e9
    ref = (lg > lg.gather(1, tg[:, None])).sum(1) + 1
    r1 = ops.sasrec_rank(m._binding(seqs), seqs, tg)
    assert torch.equal(r1, ref)
    assert torch.equal(rank_batch(m, seqs, tg), ref)
    ref0 = (logits > logits.gather(1, tg[:, None])).sum(1) + 1
    assert torch.equal(ops.sasrec_rank(m._binding(seqs), seqs, tg, mask_col0=False), ref0)
    # a target outside the table raises IndexError at the next check (evaluate.py:30's gather would)
    ops.check_errors(dev)
    bad = tg.clone()
    bad[-1] = items + 5
    ops.sasrec_rank(m._binding(seqs), seqs, bad)
    with pytest.raises(IndexError):
        ops.check_errors(dev)


def test_count_workspace_under_graph_capture(dev):
    """score_count_gt's zero-on-entry workspace stays correct across a captured call,
    its replays, eager calls on the same stream and a second capture."""
    from gr_amd import ops
    g = torch.Generator().manual_seed(77)
    h = torch.randn(200, 64, generator=g).to(dev)
    t = torch.randn(5000, 64, generator=g).to(dev)
    thr = torch.randn(200, generator=g).to(dev)
    ref = (ops.score(h, t) > thr[:, None]).sum(1)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        graphs, outs = [], []
        for _ in range(2):
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                outs.append(ops.score_count_gt(h, t, thr, mask_col0=False))
            graphs.append(gr)
            for _ in range(3):
                gr.replay()
                s.synchronize()
                assert torch.equal(outs[-1], ref)
                assert torch.equal(ops.score_count_gt(h, t, thr, mask_col0=False), ref)   # eager, same stream
        graphs[0].replay()
        s.synchronize()
        assert torch.equal(outs[0], ref)
    torch.cuda.current_stream(dev).wait_stream(s)
    assert torch.equal(ops.score_count_gt(h, t, thr, mask_col0=False), ref)


@pytest.mark.parametrize("name", ["sas_csv_c1", "sas_syn_c3", "sas_syn_c5"])
def test_fused_rank_matches_fixture(name, dev):
    from gr_amd import SASRec, ops
    from gr_amd.evaluate import hr_ndcg
    sd, out, meta = gl.load(name)
    p = dict(meta["params"], device=str(dev))
    m = SASRec(meta["item_num"], p)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev).eval()
    seqs = torch.from_numpy(out["seqs"]).to(dev)
    tg = torch.from_numpy(out["targets"]).to(dev)
    h = m.last_hidden(seqs)
    assert meta["params"]["d"] in (16, 32, 64, 128)   # the fused rank's widths (d = 16: SASRec/main.py:12)
    ranks = ops.score_rank(h, m.item_emb.weight, tg).cpu().numpy()
    ref = ops.rank(m.predict(seqs), tg).cpu().numpy()
    assert np.array_equal(ranks, ref)
    cert = out["margin"] > 1e-5
    assert np.array_equal(ranks[cert], out["ranks"][cert])
    assert hr_ndcg(ranks, 10) == (meta["hr10"], pytest.approx(meta["ndcg10"], abs=0, rel=0))


def test_evaluate_harness_config1(dev, tmp_path):
    """SASRec/evaluate.py end to end on the config-1 data: dataset from the stu-major interactions,
    checkpoint from the fixture's state dict (weights_only load), fused and materialised ranks."""
    from gr_amd.data import SASRecDataset
    from gr_amd.evaluate import evaluate
    from test_data import c1_fixture_perm, c1_records
    sd, out, meta = gl.load("sas_csv_c1")
    recs = c1_records()
    params = dict(meta["params"], device=str(dev), eval_batch_size=5, top_k=10, topk_list=[2, 5, 10, 20],
                  min_seq_len=3, ckpt=str(tmp_path / "c1.pt"), params_path=str(tmp_path / "res.csv"),
                  task_id="c1")
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, params["ckpt"])
    ds = SASRecDataset(recs, max_len=params["max_len"], mode="test", params=params)
    res, ranks = evaluate(params, dataset=ds)
    assert np.array_equal(ranks, out["ranks"][c1_fixture_perm(ds.user_ids)])
    assert res["Hit@10"] == meta["hr10"]
    assert list(res) == ["Hit@10", "NDCG@10"]            # evaluate.py:51: exactly these two keys
    res2, ranks2, multi = evaluate(params, dataset=ds, materialize=True, save_csv=False, with_multi_k=True)
    assert np.array_equal(ranks2, ranks) and res2 == res
    assert sorted(multi) == sorted(f"{m}@{k}" for k in (2, 5, 10, 20) for m in ("Hit", "NDCG"))
    # the CSV row of evaluate.py:57-89: task_id, the hyper-parameters present in params, then
    # Hit@top_k / NDCG@top_k at 6 decimals -- no multi-k columns
    import csv
    with open(params["params_path"], newline="", encoding="utf-8") as f:
        rows = list(csv.reader(f))
    hp = [k for k in ["d", "num_blocks", "num_heads", "dropout", "lr", "batch_size", "epochs",
                      "mlp_layer", "max_len", "top_k"] if k in params]
    assert rows[0] == ["task_id"] + hp + ["Hit@10", "NDCG@10"]
    assert len(rows) == 2
    assert rows[1][0] == "c1" and rows[1][-2:] == [f"{res['Hit@10']:.6f}", f"{res['NDCG@10']:.6f}"]


def test_train_evaluate_valid_mask(dev):
    """SASRec/train.py:33-56 on the GPU kernels: target-0 users dropped, multi-k metrics over the
    rest equal to the fixture ranks' (certified users)."""
    from gr_amd import SASRec
    from gr_amd.evaluate import multi_k, train_evaluate
    sd, out, meta = gl.load("sas_syn_c3")
    m = SASRec(meta["item_num"], dict(meta["params"], device=str(dev)))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    m = m.to(dev)
    seqs = torch.from_numpy(out["seqs"])
    tg = torch.from_numpy(out["targets"]).clone()
    tg[::3] = 0
    loader = [(seqs[i:i + 50], tg[i:i + 50]) for i in range(0, len(seqs), 50)]
    params = {"topk_list": [2, 5, 10, 20]}
    hk, nk = train_evaluate(m, loader, params, dev)
    assert m.training
    keep = tg.numpy() != 0
    m.eval()
    # train.py:44-48 run as written on the GPU's own logits, target-0 users removed first
    logits = m.predict(seqs[keep].to(dev))
    logits[:, 0] = -1e9
    t = torch.from_numpy(out["targets"][keep]).to(dev)
    ranks = ((logits > logits.gather(1, t[:, None])).sum(1) + 1).cpu().numpy()
    cert = out["margin"][keep] > 1e-5
    assert np.array_equal(ranks[cert], out["ranks"][keep][cert])
    ref_h, ref_n = multi_k(ranks, params["topk_list"])
    assert hk == ref_h and nk == ref_n
    assert multi_k(ranks, params["topk_list"]) == multi_k(
        np.concatenate([ranks, [1, 1]]), params["topk_list"], np.concatenate([out["targets"][keep], [0, 0]]))


def test_bad_ids_raise_without_check_mode(dev):
    """with GR_AMD_CHECK off (the default), an out-of-range item id still raises
    IndexError at the end of evaluate() (sticky device error word, one sync per evaluation)."""
    from gr_amd import SASRec, ops
    from gr_amd.data import SASRecDataset
    from gr_amd.evaluate import evaluate
    assert not ops.CHECK
    sd, out, meta = gl.load("sas_csv_c1")
    m = SASRec(meta["item_num"], dict(meta["params"], device=str(dev)))
    m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    recs = [("u1", [1, 2, 3]), ("u2", [4, meta["item_num"] + 5, 6])]
    ds = SASRecDataset(recs, max_len=meta["params"]["max_len"], mode="test", params={"min_seq_len": 3})
    params = dict(meta["params"], device=str(dev), top_k=10)
    with pytest.raises(IndexError):
        evaluate(params, dataset=ds, model=m.to(dev), save_csv=False)
    ops.check_errors(dev)          # the flag was cleared by the raise
