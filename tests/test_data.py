"""Host-side input formats and the evaluation tail's metric semantics."""
import csv
import json
import os

import numpy as np
import pytest
import torch

import golden_lib as gl
from gr_amd.data import EmbDataset, SASRecDataset, read_interactions, reference_order
from gr_amd.evaluate import hr_ndcg, multi_k, save_results_to_csv


def c1_records():
    """The config-1 interactions in the reference's h5 order (ORDER BY student_id, id)."""
    z = np.load(os.path.join(gl.HERE, "interactions_c1.npz"), allow_pickle=False)
    rows = reference_order(list(zip(z["student_id"].tolist(), z["row_id"].tolist(), z["class_id"].tolist())))
    return [(s, [int(c)]) for s, _, c in rows]


def c1_fixture_perm(user_ids):
    """Row permutation from the C1 fixture (users in first-seen FILE order, make_golden.py) to
    ``user_ids``: per-user outputs are compared after it."""
    z = np.load(os.path.join(gl.HERE, "interactions_c1.npz"), allow_pickle=False)
    seen = {}
    for s in z["student_id"].tolist():
        seen[s] = seen.get(s, 0) + 1
    file_users = [u for u, c in seen.items() if c >= 3]
    return np.array([file_users.index(u) for u in user_ids])


def test_sasrec_test_dataset_matches_config1_fixture():
    """stu-major interactions -> per-user test sequences: the inputs / targets / item_num the C1
    golden fixture was generated with (SASRec/data_vision.py:16-38, 74-87), users in the order of
    the reference's h5 file (Baseline/data_process.py:22-27)."""
    _, out, meta = gl.load("sas_csv_c1")
    ds = SASRecDataset(c1_records(), max_len=20, mode="test", params={"min_seq_len": 3})
    inp, tgt = ds.tensors()
    assert ds.item_num == meta["item_num"]
    assert ds.user_ids == sorted(ds.user_ids, key=lambda u: u.encode())
    perm = c1_fixture_perm(ds.user_ids)
    assert np.array_equal(inp.numpy(), out["seqs"][perm]) and np.array_equal(tgt.numpy(), out["targets"][perm])
    x, t = ds[3]
    assert torch.equal(x, inp[3]) and int(t) == int(tgt[3])
    b = list(ds.batches(5))
    assert len(b) == 4 and torch.equal(torch.cat([p[0] for p in b]), inp)


def test_sasrec_dataset_semantics():
    recs = [("u2", [5, 6]), ("u1", [1, 2, 3]), ("u2", [7]), ("u3", [9, 1]), ("u4", [2, 3, 4, 5, 6])]
    ds = SASRecDataset(recs, max_len=3, mode="test", params={"min_seq_len": 3})
    assert ds.user_ids == ["u2", "u1", "u4"]                 # first-seen order, u3 too short
    assert ds.item_num == 9                                  # max over ALL users (data_vision.py:36-38)
    inp, tgt = ds.tensors()
    assert inp.tolist() == [[0, 5, 6], [0, 1, 2], [3, 4, 5]] and tgt.tolist() == [7, 3, 6]
    tr = SASRecDataset(recs, max_len=4, mode="train", params={"min_seq_len": 3})
    x, y = tr[2]                                             # u4: train seq [2,3,4,5]
    assert x.tolist() == [0, 2, 3, 4] and y.tolist() == [0, 3, 4, 5]


def test_interaction_and_embedding_csv_readers(tmp_path):
    p = tmp_path / "inter.csv"
    vec = [0.5] * 4
    with open(p, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["id", "student_id", "class_id", "bert_vector"])
        w.writerow([1, "a", 3, json.dumps(vec)])
        w.writerow([2, "", 4, json.dumps(vec)])
        w.writerow([3, "b", 5, json.dumps([1.0] * 4)])
    assert read_interactions(str(p)) == [("a", [3]), ("b", [5])]
    q = tmp_path / "unordered.csv"      # SQL ORDER BY student_id, id: bytewise ids, then row id
    with open(q, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(["id", "student_id", "class_id"])
        for rid, sid, cid in [(5, "b", 1), (2, "a", 2), (9, "B", 3), (1, "b", 4), (3, "a", 5)]:
            w.writerow([rid, sid, cid])
    assert read_interactions(str(q)) == [("B", [3]), ("a", [2]), ("a", [5]), ("b", [4]), ("b", [1])]
    e = EmbDataset(str(p))
    assert e.embeddings.shape == (2, 4) and e.dim == 4 and e.embeddings.dtype == np.float32
    np.save(tmp_path / "e.npy", np.arange(12, dtype=np.float32).reshape(3, 4))
    e2 = EmbDataset(str(tmp_path / "e.npy"))
    assert len(e2) == 3 and torch.equal(e2[1], torch.tensor([4.0, 5, 6, 7]))
    assert [b.shape[0] for b in e2.batches(2)] == [2, 1]


def test_h5_needs_h5py_message(tmp_path):
    try:
        import h5py  # noqa: F401
        pytest.skip("h5py present")
    except ImportError:
        pass
    with pytest.raises(ImportError, match="h5py"):
        read_interactions(str(tmp_path / "x.h5"))


def test_metrics_match_reference_tail(tmp_path):
    """HR/NDCG exactly as evaluate.py:35-47 / train.py:33-56 (float64 np.mean of per-user lists)."""
    ranks = np.array([1, 3, 10, 11, 2, 50, 7], np.int64)
    hit, ndcg = hr_ndcg(ranks, 10)
    ref_h = np.mean([1 if r <= 10 else 0 for r in ranks])
    ref_n = np.mean([1 / np.log2(r + 1) if r <= 10 else 0 for r in ranks])
    assert hit == ref_h and ndcg == ref_n
    hk, nk = multi_k(ranks, [2, 5, 10, 20])
    assert hk[10] == hit and nk[10] == ndcg and hk[2] == np.mean([1, 0, 0, 0, 1, 0, 0])
    params = {"params_path": str(tmp_path / "r.csv"), "task_id": "t", "d": 16, "top_k": 10}
    save_results_to_csv(params, {"Hit@10": hit, "NDCG@10": ndcg})
    save_results_to_csv(params, {"Hit@10": hit, "NDCG@10": ndcg})
    rows = list(csv.reader(open(params["params_path"])))
    assert rows[0] == ["task_id", "d", "top_k", "Hit@10", "NDCG@10"] and len(rows) == 3
    assert rows[1][3] == f"{hit:.6f}"


def test_metric_arrays_equal_reference_loops():
    """hr_ndcg / multi_k build the reference's per-user lists as arrays (one scalar log2 per distinct
    rank): bitwise the loops of evaluate.py:36-47 and train.py:46-53 on many rank vectors."""
    rng = np.random.default_rng(5)
    for n, hi in [(1, 3), (7, 12), (1000, 30), (95_423, 800), (4096, 11), (50_000, 100_000)]:
        ranks = rng.integers(1, hi, n)
        for top_k in (1, 2, 5, 10, 20):
            ht, nd = [], []
            for r in ranks:
                if r <= top_k:
                    ht.append(1)
                    nd.append(1 / np.log2(r + 1))
                else:
                    ht.append(0)
                    nd.append(0)
            assert hr_ndcg(ranks, top_k) == (float(np.mean(ht)), float(np.mean(nd)))
        hk, nk = multi_k(ranks, [2, 5, 10, 20])
        for k in (2, 5, 10, 20):
            assert nk[k] == float(np.mean([1 / np.log2(r + 1) if r <= k else 0 for r in ranks]))
            assert hk[k] == float(np.mean([1 if r <= k else 0 for r in ranks]))


def test_multi_k_drops_target_zero_users():
    """train.py:42-45: users with target 0 are removed before ranking (valid_mask)."""
    ranks = np.array([1, 3, 10, 11, 2], np.int64)
    targets = np.array([5, 0, 7, 0, 9], np.int64)
    hk, nk = multi_k(ranks, [2, 10], targets)
    assert hk[2] == np.mean([1, 0, 1]) and hk[10] == 1.0
    assert nk[10] == np.mean([1.0, 1 / np.log2(11), 1 / np.log2(3)])
