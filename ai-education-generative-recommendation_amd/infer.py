"""Semantic-ID emission of RQ-VAE/infer.py:44-184 on the gfx950 kernels.

1. codes of every item with ``get_indices(use_sk=False)`` in the reference's batch-64 DataLoader
   call pattern (``RQVAE.get_indices_batched``): MKL's CPU order depends on a call's row count, and
   a tail batch of 1-15 rows (707 items: 3) takes its small-call order, so the tail is its own call;
   the full batches share one launch;
2. collision rounds (infer.py:108-130): every level but the last gets ``sk_epsilon = 0`` (the
   reference mutates the model the same way), then up to 30 times: group the items that share a
   code (first-appearance order, infer.py:29-41) and re-encode each group with ``use_sk=True`` —
   all groups of a round in ONE launch, one workgroup per group (``RQVAE.get_indices_groups``);
3. dedup digit (infer.py:139-162): append a zero column and number the members of every code that
   is still shared;
4. ``np.save`` of the (N, L+1) code array and the ``_mapping.json`` index -> code table
   (infer.py:164-184).
"""
import collections
import json
import os

import numpy as np
import torch

from .data import EmbDataset


def collision_groups(codes):
    """get_collision_item (infer.py:29-41): groups of rows sharing a code, in order of the code's
    first appearance, members in row order."""
    index2id = collections.OrderedDict()
    for i, c in enumerate(map(tuple, np.asarray(codes).tolist())):
        index2id.setdefault(c, []).append(i)
    return [g for g in index2id.values() if len(g) > 1]


def dedup_codes(codes):
    """infer.py:139-162: zero column appended, then 0, 1, 2, ... for the members of each shared code."""
    codes_array = np.hstack((np.asarray(codes), np.zeros((len(codes), 1), dtype=int)))
    unique_codes, counts = np.unique(codes_array, axis=0, return_counts=True)
    for duplicate in unique_codes[counts > 1]:
        for i, idx in enumerate(np.where((codes_array == duplicate).all(axis=1))[0]):
            codes_array[idx, -1] = i
    return codes_array


@torch.no_grad()
def generate_codes(model, embeddings, device, max_rounds=30, log=None, batch_size=64):
    """Steps 1-3 for ``embeddings`` [N, in_dim] (numpy or tensor).  Returns (codes [N, L] after the
    collision rounds, codes_array [N, L+1] with the dedup digit, stats).  ``batch_size``: the
    reference DataLoader's (infer.py:85)."""
    x = torch.as_tensor(np.asarray(embeddings, dtype=np.float32) if not torch.is_tensor(embeddings)
                        else embeddings, dtype=torch.float32).to(device)
    codes = model.get_indices_batched(x, batch_size).cpu().numpy()
    for vq in model.rq.vq_layers[:-1]:                        # infer.py:109-110
        vq.sk_epsilon = 0.0
    rounds = 0
    for _ in range(max_rounds):
        groups = collision_groups(codes)
        if not groups:
            break
        if log:
            log(f"Iteration {rounds}: Found {len(groups)} collision groups")
        rows = np.concatenate(groups)
        out = model.get_indices_groups(x[torch.from_numpy(rows).to(device)], [len(g) for g in groups])
        codes[rows] = out.cpu().numpy()
        rounds += 1
    counts = collections.Counter(map(tuple, codes.tolist()))
    tot = len(codes)
    stats = {"rounds": rounds, "max_conflicts": max(counts.values()) if tot else 0,
             "collision_rate": (tot - len(counts)) / tot if tot else 0.0}
    return codes, dedup_codes(codes), stats


def save_codes(codes_array, output_file):
    """infer.py:164-184: ``<output_file>`` (.npy) and ``<output_file minus .npy>_mapping.json``."""
    os.makedirs(os.path.dirname(output_file) or ".", exist_ok=True)
    np.save(output_file, codes_array)
    mapping_file = output_file.replace(".npy", "_mapping.json")
    with open(mapping_file, "w") as f:
        json.dump({i: code.tolist() for i, code in enumerate(codes_array)}, f, indent=2)
    return mapping_file


def infer(params, model=None, data=None, log=print):
    """RQ-VAE/infer.py:infer(params) with the same params keys (RQ-VAE/main.py:4-33).  The
    checkpoint ``<ckpt_dir>/best_collision_model.pth`` is read with ``weights_only=True`` (a
    reference checkpoint also pickles its args dict; pass ``model=`` to use an already-loaded
    one)."""
    from .rqvae import RQVAE
    device = torch.device(params["device"])
    if data is None:
        data = EmbDataset(params["data_path"])
    if model is None:
        model = RQVAE(in_dim=data.dim, num_emb_list=params["num_emb_list"], e_dim=params["e_dim"],
                      layers=params["layers"], dropout_prob=params["dropout"],
                      bn=params["batch_normalize"], loss_type=params["loss_type"],
                      quant_loss_weight=params["quant_loss_weight"],
                      kmeans_init=params["kmeans_init"], kmeans_iters=params["kmeans_iters"],
                      sk_epsilons=params["sk_epsilons"], sk_iters=params["sk_iters"])
        ckpt_path = os.path.join(params["ckpt_dir"], "best_collision_model.pth")
        if os.path.exists(ckpt_path):
            ckpt = torch.load(ckpt_path, map_location="cpu", weights_only=True)
            model.load_state_dict(ckpt["state_dict"] if "state_dict" in ckpt else ckpt)
        elif log:
            log(f"Warning: No checkpoint found at {ckpt_path}, using randomly initialized model")
    model = model.to(device).eval()
    codes, codes_array, stats = generate_codes(model, data.embeddings, device, log=log)
    if log:
        log(f"All indices number: {len(codes)}; max conflicts {stats['max_conflicts']}; "
            f"collision rate {stats['collision_rate']}")
    save_codes(codes_array, params["semantic_id_file"])
    return codes_array, stats
