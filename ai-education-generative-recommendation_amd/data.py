"""Input formats of the two hot paths: host-side loaders that produce
exactly the tensors the reference's datasets hand to the models.

* ``SASRecDataset`` — SASRec/data_vision.py:7-87.  Interaction records (user_id, item sequence)
  grouped per user in first-seen order (``defaultdict``, :16-19), users shorter than
  ``min_seq_len`` dropped (:24), ``item_num`` = the largest item id over ALL users (:36-38).
  ``mode='test'``: input = the last ``max_len`` items of ``seq[:-1]`` left-padded with 0, target =
  ``seq[-1]`` (:74-87); ``mode='train'``: shifted input/target pairs (:56-72).
* ``EmbDataset`` — RQ-VAE/vision_data.py:9-30: ``item_embs`` [N, 768] float32 (+ ``meta``).

Sources: h5 (the reference's format; needs ``h5py``, which is optional and imported lazily),
``.npz`` with the same dataset names, plain ``.npy`` embeddings, or an interaction CSV such as
stu-major/interaction_records.csv (``student_id``, ``class_id``; rows without a student are
skipped and the rest ordered by (student_id, id) exactly as Baseline/data_process.py:22-27's
``ORDER BY student_id, id`` builds the reference's h5 file, so users come out in that order).
Batches are built on the host as whole tensors (no per-item Python ``__getitem__`` calls) and moved
to the GPU by the caller, as in SASRec/evaluate.py:21-23.
"""
import csv
import json
import os
from collections import OrderedDict

import numpy as np
import torch


def _h5():
    try:
        import h5py  # noqa: F401
        return h5py
    except ImportError as e:   # the reference needs it too; say so plainly
        raise ImportError("reading the reference's .h5 files needs h5py, which is not installed; "
                          "convert the file to .npz (same dataset names) or pass arrays") from e


def read_interactions(path):
    """[(user_id, [item ids...])] in file order from .h5 / .npz (``user_id``, ``item_id_list``) or
    an interaction CSV (``student_id``, ``class_id``: one row per interaction)."""
    ext = os.path.splitext(path)[1].lower()
    if ext in (".h5", ".hdf5"):
        with _h5().File(path, "r") as f:                       # data_vision.py:40-46
            users = f["user_id"][:]
            items = f["item_id_list"][:]
        return [(u, [int(i) for i in seq]) for u, seq in zip(users, items)]
    if ext == ".npz":
        z = np.load(path, allow_pickle=False)
        users = z["user_id"]
        if "item_id_list" in z:                                  # padded [U, L] with lengths
            lens = z["item_len"]
            return [(u, [int(i) for i in row[:n]]) for u, row, n in zip(users, z["item_id_list"], lens)]
        raise KeyError(f"{path}: expected user_id / item_id_list / item_len arrays")
    if ext == ".csv":
        rows = []
        with open(path, encoding="utf-8-sig", newline="") as f:
            for k, row in enumerate(csv.DictReader(f)):
                s = (row.get("student_id") or "").strip()
                if s:
                    rid = int(row["id"]) if (row.get("id") or "").strip() else k
                    rows.append((s, rid, int(row["class_id"])))
        return [(s, [c]) for s, _, c in reference_order(rows)]
    raise ValueError(f"unsupported interaction file: {path}")


def reference_order(rows):
    """Stable sort of (student_id, id, ...) interaction rows by ``ORDER BY student_id, id``
    (Baseline/data_process.py:22-27): SQLite compares TEXT student ids bytewise (BINARY collation on
    UTF-8), then the integer row id."""
    return sorted(rows, key=lambda r: (str(r[0]).encode("utf-8"), int(r[1])))


class SASRecDataset:
    """SASRec/data_vision.py:SASRecDataset over records [(user_id, items)] or a file path."""

    def __init__(self, records, max_len=50, mode="train", params=None):
        if isinstance(records, (str, os.PathLike)):
            records = read_interactions(records)
        self.max_len = max_len
        self.mode = mode
        self.params = params or {}
        hist = OrderedDict()
        for user_id, seq in records:                             # data_vision.py:16-19
            hist.setdefault(user_id, []).extend(int(i) for i in seq)
        self.user_ids = []
        self.user_seqs = []
        for user_id, items in hist.items():
            if len(items) < self.params.get("min_seq_len", 3):   # :24
                continue
            if mode == "train":
                if len(items[:-1]) >= 1:
                    self.user_seqs.append(items[:-1])
                    self.user_ids.append(user_id)
            elif mode == "test":
                self.user_seqs.append(items)
                self.user_ids.append(user_id)
            else:
                raise ValueError(f"mode must be 'train' or 'test', got {mode!r}")
        all_items = [i for items in hist.values() for i in items]
        self.item_num = max(all_items) if all_items else 0       # :36-38

    def __len__(self):
        return len(self.user_seqs)

    def __getitem__(self, idx):
        inp, tgt = self._one(self.user_seqs[idx])
        return torch.tensor(inp, dtype=torch.long), torch.tensor(tgt, dtype=torch.long)

    def _one(self, seq):
        n = self.max_len
        if self.mode == "train":                                 # :56-72
            raw_in, raw_tg = seq[:-1][-n:], seq[1:][-n:]
            pad = n - len(raw_in)
            return [0] * pad + raw_in, [0] * pad + raw_tg
        if len(seq) < 2:                                         # :76-77
            return [0] * n, 0
        inp = seq[:-1]
        s = inp[-n:] if len(inp) >= n else [0] * (n - len(inp)) + inp
        return s, seq[-1]

    def tensors(self):
        """The whole dataset as (inputs [U, n] int64, targets [U] or [U, n] int64)."""
        pairs = [self._one(s) for s in self.user_seqs]
        inp = torch.tensor([p[0] for p in pairs], dtype=torch.long).reshape(len(pairs), self.max_len)
        tgt = torch.tensor([p[1] for p in pairs], dtype=torch.long)
        return inp, tgt

    def batches(self, batch_size):
        """DataLoader(shuffle=False) equivalent: consecutive (inputs, targets) batches."""
        inp, tgt = self.tensors()
        for i in range(0, len(inp), batch_size):
            yield inp[i:i + batch_size], tgt[i:i + batch_size]


class EmbDataset:
    """RQ-VAE/vision_data.py:EmbDataset: ``item_embs`` [N, dim] float32 (+ optional ``meta``)."""

    def __init__(self, path_or_array):
        self.meta = {}
        if isinstance(path_or_array, (str, os.PathLike)):
            self.path = str(path_or_array)
            self.embeddings = self._load(self.path)
        else:
            self.path = None
            self.embeddings = np.ascontiguousarray(np.asarray(path_or_array, dtype=np.float32))
        self.dim = self.embeddings.shape[-1]

    def _load(self, path):
        ext = os.path.splitext(path)[1].lower()
        if ext in (".h5", ".hdf5"):
            with _h5().File(path, "r") as f:                      # vision_data.py:17-22
                emb = f["item_embs"][:]
                if "meta" in f:
                    self.meta = json.loads(f["meta"][()].decode("utf-8"))
            return np.ascontiguousarray(emb, dtype=np.float32)
        if ext == ".npz":
            z = np.load(path, allow_pickle=False)
            if "meta" in z:
                self.meta = json.loads(str(z["meta"]))
            return np.ascontiguousarray(z["item_embs"], dtype=np.float32)
        if ext == ".npy":
            return np.ascontiguousarray(np.load(path, allow_pickle=False), dtype=np.float32)
        if ext == ".csv":                                         # stu-major bert_vector column
            with open(path, encoding="utf-8-sig", newline="") as f:
                rows = [r for r in csv.DictReader(f) if (r.get("student_id") or "").strip()]
            return np.array([json.loads(r["bert_vector"]) for r in rows], dtype=np.float64).astype(np.float32)
        raise ValueError(f"unsupported embedding file: {path}")

    def __len__(self):
        return len(self.embeddings)

    def __getitem__(self, index):
        return torch.from_numpy(np.ascontiguousarray(self.embeddings[index]))

    def batches(self, batch_size):
        """DataLoader(shuffle=False) equivalent over the embedding rows."""
        for i in range(0, len(self.embeddings), batch_size):
            yield torch.from_numpy(self.embeddings[i:i + batch_size])
