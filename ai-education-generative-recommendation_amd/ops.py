"""Tensor-level wrappers of the C ABI (include/gr_amd.h).

Each function takes/returns torch tensors on a ROCm device, enqueues on the current stream and
never synchronises.  Argument checking mirrors the ATen errors the reference would raise.
"""
import ctypes
import itertools
import os

import torch

from . import _lib as L

# Input errors the kernels detect (an item id outside the table, a row whose negatives cannot be
# drawn) are OR-ed into a per-device sticky error word instead of synchronising the stream.
# ``check_errors()`` synchronises and raises (evaluate() calls it once per evaluation; a training
# loop calls it once per epoch).  GR_AMD_CHECK=1 checks after every call instead.
CHECK = os.environ.get("GR_AMD_CHECK", "0") == "1"
ERR_BAD_ID = 1        # item id outside [0, rows): the reference raises IndexError (nn.Embedding / gather)
ERR_NEG_POPULATION = 2  # get_neg_samples population smaller than num_neg: numpy raises ValueError
_ERR = {}


def err_flag(device):
    """The device's sticky error word (int32, 0 = clean); kernels only ever write a nonzero code."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _ERR.get(idx)
    if t is None:
        t = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", idx))
        _ERR[idx] = t
    return t


def check_errors(device=None):
    """Synchronise ``device`` and raise the error the kernels flagged since the last check (then
    clear it): IndexError for out-of-range item ids, ValueError for an unfillable negative row."""
    devs = [device] if device is not None else [torch.device("cuda", i) for i in list(_ERR)]
    for d in devs:
        t = err_flag(torch.device(d))
        code = int(t.item())              # .item() synchronises the stream the flag was written on
        if code:
            t.zero_()
            if code == ERR_NEG_POPULATION:
                raise ValueError("Cannot take a larger sample than population when 'replace=False'")
            raise IndexError("index out of range in self (item id outside the embedding table)")


def linear(x, weight, bias=None, act="none", residual=None, out=None):
    """``act(x @ weight.T + bias) (+ residual)`` — F.linear (+ the activations of
    RQ-VAE/models/layers.py:45-67: relu, sigmoid, tanh, leakyrelu) on the matrix cores."""
    L.require_gpu(x, weight)
    x2 = L.as_f32(x).reshape(-1, x.shape[-1])
    w = L.as_f32(weight)
    m, k = x2.shape
    n = w.shape[0]
    if w.shape[1] != k:
        raise RuntimeError(f"linear: shape mismatch x[..., {k}] vs weight{tuple(w.shape)}")
    b = L.as_f32(bias) if bias is not None else None
    r = L.as_f32(residual).reshape(m, n) if residual is not None else None
    y = out if out is not None else torch.empty((m, n), dtype=torch.float32, device=x.device)
    a = {"none": L.GR_ACT_NONE, "relu": L.GR_ACT_RELU, "sigmoid": L.GR_ACT_SIGMOID, "tanh": L.GR_ACT_TANH,
         "leakyrelu": L.GR_ACT_LEAKYRELU}[act]
    with L.on(x.device):
        L.check(L.lib().gr_linear_f32(L.ptr(x2), m, k, L.ptr(w), n, L.ptr(b), L.ptr(r),
                                      n if r is not None else 0, a, L.ptr(y), n,
                                      L.stream_of(x.device)), "gr_linear_f32")
    return y.reshape(*x.shape[:-1], n)


def score(h, table, out=None):
    """Full-catalog logits ``h @ table.T`` (SASRec/model.py:107)."""
    L.require_gpu(h, table)
    h = L.as_f32(h)
    t = L.as_f32(table)
    B, d = h.shape
    rows = t.shape[0]
    y = out if out is not None else logits_buffer(B, rows, h.device)
    with L.on(h.device):
        L.check(L.lib().gr_score_f32(L.ptr(h), B, d, L.ptr(t), rows, L.ptr(y), y.stride(0),
                                     L.stream_of(h.device)), "gr_score_f32")
    return y


def rank(logits, targets, mask_col0=True):
    """Strict rank of each target (SASRec/evaluate.py:27-32) without mutating ``logits``."""
    L.require_gpu(logits, targets)
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    t = targets.reshape(-1).to(torch.int64).contiguous()
    B, cols = logits.shape
    out = torch.empty(B, dtype=torch.int64, device=logits.device)
    with L.on(logits.device):
        L.check(L.lib().gr_rank_f32(L.ptr(logits), B, cols, logits.stride(0), L.ptr(t),
                                    1 if mask_col0 else 0, L.ptr(out),
                                    L.stream_of(logits.device)), "gr_rank_f32")
    return out


def count_gt(logits, thresholds):
    """``#{j : logits[b, j] > thresholds[b]}`` per row (strict, SASRec/evaluate.py:32)."""
    L.require_gpu(logits, thresholds)
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    th = L.as_f32(thresholds.reshape(-1))
    B, cols = logits.shape
    out = torch.empty(B, dtype=torch.int64, device=logits.device)
    with L.on(logits.device):
        L.check(L.lib().gr_count_gt_f32(L.ptr(logits), B, cols, logits.stride(0), L.ptr(th),
                                        L.ptr(out), L.stream_of(logits.device)), "gr_count_gt_f32")
    return out


def topk(logits, k, id_offset=0, thresholds=None):
    """Per-row top-k: (values [B,k] descending, ids [B,k] = column + id_offset); ties -> lower id.
    With ``thresholds`` the same pass also returns the strict counts ``#{j : l[b,j] > thr[b]}``."""
    L.require_gpu(logits)
    if logits.stride(1) != 1:
        logits = logits.contiguous()
    B, cols = logits.shape
    dev = logits.device
    vals = torch.empty((B, k), dtype=torch.float32, device=dev)
    ids = torch.empty((B, k), dtype=torch.int64, device=dev)
    th = L.as_f32(thresholds.reshape(-1)) if thresholds is not None else None
    cnt = torch.empty(B, dtype=torch.int64, device=dev) if th is not None else None
    nbytes = L.lib().gr_topk_workspace_bytes(B, cols, k)
    wsp = L.workspace(nbytes, dev)
    with L.on(dev):
        L.check(L.lib().gr_topk_f32(L.ptr(logits), B, cols, logits.stride(0), k, id_offset,
                                    L.ptr(vals), L.ptr(ids), L.ptr(th), L.ptr(cnt), L.ptr(wsp), nbytes,
                                    L.stream_of(dev)), "gr_topk_f32")
    return (vals, ids) if th is None else (vals, ids, cnt)


def score_pairs(h, table, ids, mask_col0=True):
    """Target logits ``h[b] . table[ids[b]]`` with the scoring kernel's exact fp32 chain (-1e9 for
    id 0 when ``mask_col0``, SASRec/evaluate.py:27)."""
    L.require_gpu(h, table, ids)
    h, t = L.as_f32(h), L.as_f32(table)
    ids = ids.reshape(-1).to(torch.int64).contiguous()
    B, d = h.shape
    out = torch.empty(B, dtype=torch.float32, device=h.device)
    err = err_flag(h.device)
    with L.on(h.device):
        L.check(L.lib().gr_score_pairs_f32(L.ptr(h), B, d, L.ptr(t), t.shape[0], L.ptr(ids),
                                           1 if mask_col0 else 0, L.ptr(out), L.ptr(err),
                                           L.stream_of(h.device)), "gr_score_pairs_f32")
    _check_err(err)
    return out


_COUNT_WS = {}   # (device, stream) -> zeroed workspace of gr_score_count_gt_ws_f32 (left zero by every call)
_SCRATCH = {}    # (device index, stream) -> scratch workspace of the short calls (no contents carried)
SCRATCH_CACHE_BYTES = 16 << 20


def scratch(nbytes, device):
    """Caller-owned scratch for one call (``L.workspace``), reused across the calls of one stream when
    small: a call's kernels finish with it before any later call on the same stream starts (stream
    order), and the library never keeps pointers.  Saves an allocation per call at the reference's
    batch sizes (get_indices(x[64]), rank of 128 users).  Under graph capture: a fresh allocation
    (the graph's pool owns it)."""
    if nbytes > SCRATCH_CACHE_BYTES or torch.cuda.is_current_stream_capturing():
        return L.workspace(nbytes, device)
    key = (device.index, L.stream_of(device))
    ws = _SCRATCH.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = L.workspace(max(nbytes, 1 << 16), device)
        _SCRATCH[key] = ws
    return ws


def _count_workspace(device, nbytes):
    """The count kernel's workspace, which it expects zero on entry and leaves zero on exit.
    Eager calls reuse one cached, once-zeroed buffer per (device, stream).  Under graph capture a
    fresh buffer is allocated and zeroed by a node of the graph itself, and never cached: a cached
    buffer first zeroed inside a capture holds zeros only after a replay, and the capture stream's
    key is reused by later captures."""
    if torch.cuda.is_current_stream_capturing():
        # zeroed by a fill KERNEL node of the graph (torch.zeros), so every replay starts from zeros
        return torch.zeros(nbytes, dtype=torch.uint8, device=device), None
    key = (device, torch.cuda.current_stream(device).cuda_stream)
    ws = _COUNT_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        _COUNT_WS[key] = ws
    return ws, key


def score_count_gt(h, table, thresholds, mask_col0=True):
    """``#{j : (h . table^T)[b, j] > thresholds[b]}`` without materialising the logits."""
    L.require_gpu(h, table, thresholds)
    h, t = L.as_f32(h), L.as_f32(table)
    th = L.as_f32(thresholds.reshape(-1))
    B, d = h.shape
    out = torch.empty(B, dtype=torch.int64, device=h.device)
    with L.on(h.device):
        nb = L.lib().gr_score_count_workspace_bytes(B)
        ws, key = _count_workspace(h.device, nb)
        try:
            L.check(L.lib().gr_score_count_gt_ws_f32(L.ptr(h), B, d, L.ptr(t), t.shape[0], L.ptr(th),
                                                     1 if mask_col0 else 0, L.ptr(out), L.ptr(ws), nb,
                                                     L.stream_of(h.device)), "gr_score_count_gt_ws_f32")
        except Exception:
            if key is not None:   # a failed call may leave non-zero words: never reuse the buffer
                _COUNT_WS.pop(key, None)
            raise
    return out


def score_rank(h, table, targets, mask_col0=True):
    """Strict rank of each target over the full catalog (SASRec/evaluate.py:27-32) without
    writing the [B, rows] logits: count_gt(h, table, pairs(h, table, targets)) + 1."""
    return score_count_gt(h, table, score_pairs(h, table, targets, mask_col0), mask_col0) + 1


def score_topk(h, table, k, id_offset=0, thresholds=None, mask_col0=True):
    """Top-k of ``h @ table.T`` per user without writing the logits: (values [B,k] descending,
    ids [B,k] = column + id_offset; ties -> lower id), column 0 taken as -1e9 when ``mask_col0``
    (SASRec/evaluate.py:27).  With ``thresholds`` also the strict counts ``#{j : l[b,j] > thr[b]}``.
    Same values, bit for bit, as ``topk(score(h, table))`` after the column-0 mask."""
    L.require_gpu(h, table)
    h, t = L.as_f32(h), L.as_f32(table)
    B, d = h.shape
    rows = t.shape[0]
    dev = h.device
    vals = torch.empty((B, k), dtype=torch.float32, device=dev)
    ids = torch.empty((B, k), dtype=torch.int64, device=dev)
    th = L.as_f32(thresholds.reshape(-1)) if thresholds is not None else None
    cnt = torch.empty(B, dtype=torch.int64, device=dev) if th is not None else None
    nbytes = L.lib().gr_score_topk_workspace_bytes(B, d, rows, k)
    wsp = L.workspace(nbytes, dev)
    with L.on(dev):
        L.check(L.lib().gr_score_topk_f32(L.ptr(h), B, d, L.ptr(t), rows, id_offset,
                                          1 if mask_col0 else 0, k, L.ptr(th), L.ptr(cnt),
                                          L.ptr(vals), L.ptr(ids), L.ptr(wsp), nbytes,
                                          L.stream_of(dev)), "gr_score_topk_f32")
    return (vals, ids) if th is None else (vals, ids, cnt)


def merge_topk(vals, ids, k):
    """Top-k of candidate lists [B, C] (values, global ids) by (value desc, id asc), ids < 0 padding
    (emitted as (-inf, -1)): the merge of the catalog shards' lists (gr_merge_topk_f32)."""
    L.require_gpu(vals, ids)
    B, C = vals.shape
    v = L.as_f32(vals)
    i = ids.to(torch.int64).contiguous()
    out_v = torch.empty((B, k), dtype=torch.float32, device=vals.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=vals.device)
    with L.on(vals.device):
        L.check(L.lib().gr_merge_topk_f32(L.ptr(v), v.stride(0), L.ptr(i), i.stride(0), B, C, k,
                                          L.ptr(out_v), L.ptr(out_i), L.stream_of(vals.device)),
                "gr_merge_topk_f32")
    return out_v, out_i


def merge_topk_packed(packed, world, kk, k):
    """The merge straight from the exchange's all-gathered int64 buffer [world, B, 2 kk] (per rank
    and row kk ids, then kk value bit patterns; dist._exchange)."""
    L.require_gpu(packed)
    packed = packed.contiguous()
    B = packed.numel() // (world * 2 * kk)
    out_v = torch.empty((B, k), dtype=torch.float32, device=packed.device)
    out_i = torch.empty((B, k), dtype=torch.int64, device=packed.device)
    with L.on(packed.device):
        L.check(L.lib().gr_merge_topk_packed(L.ptr(packed), world, B, kk, k, L.ptr(out_v), L.ptr(out_i),
                                             L.stream_of(packed.device)), "gr_merge_topk_packed")
    return out_v, out_i


def rq_quantize(z, codebooks, with_gap=False):
    """Residual quantization of latents (RQ-VAE/models/rq.py:39-56, use_sk=False).

    With ``with_gap`` also returns the best distance and the best/second-best gap per level."""
    L.require_gpu(z, *codebooks)
    z = L.as_f32(z)
    n, e = z.shape
    cbs = [L.as_f32(c) for c in codebooks]
    Ks = [c.shape[0] for c in cbs]
    for c in cbs:
        if c.shape[1] != e:
            raise RuntimeError("rq_quantize: codebook width != latent width")
    dev = z.device
    idx = torch.empty((n, len(cbs)), dtype=torch.int64, device=dev)
    gap = torch.empty((n, len(cbs)), dtype=torch.float32, device=dev) if with_gap else None
    best = torch.empty((n, len(cbs)), dtype=torch.float32, device=dev) if with_gap else None
    lib = L.lib()
    st = L.stream_of(dev)
    with L.on(dev):
        # code_norms = NULL: the kernel recomputes the norms from its LDS image of each codebook
        L.check(lib.gr_rq_quantize_f32(L.ptr(z), n, e, len(cbs), L.i32_array(Ks), L.ptr_array(cbs),
                                       None, L.ptr(idx), L.ptr(best), L.ptr(gap), st),
                "gr_rq_quantize_f32")
    return (idx, best, gap) if with_gap else idx


class RqBinding:
    """The encoder weights / biases and codebooks of one RQ-VAE as the ctypes arrays
    ``gr_rq_encode_f32`` takes (device pointers, dims, K per level), built once per parameter set
    (:func:`rq_binding`) so a ``get_indices`` call at the reference's batch 64 (RQ-VAE/infer.py:84-95)
    pays only the launch."""

    def __init__(self, weights, biases, codebooks):
        weights, biases, codebooks = ([t.detach() for t in ts] for ts in (weights, biases, codebooks))
        self.ws = [L.as_f32(w) for w in weights]
        self.bs = [L.as_f32(b) for b in biases]
        self.cbs = [L.as_f32(c) for c in codebooks]
        L.require_gpu(*self.ws, *self.cbs)
        self.direct = all(a.data_ptr() == b.data_ptr() for a, b in
                          zip(self.ws + self.bs + self.cbs, list(weights) + list(biases) + list(codebooks)))
        self.in_dim = self.ws[0].shape[1]
        self.dims = [self.in_dim] + [w.shape[0] for w in self.ws]
        for i, w in enumerate(self.ws):
            if w.shape[1] != self.dims[i]:
                raise RuntimeError(f"rq_encode: Linear {i} expects {w.shape[1]} inputs, got {self.dims[i]}")
        self.Ks = [c.shape[0] for c in self.cbs]
        self.n_linear = len(self.ws)
        self.dims_c, self.ks_c = L.i32_array(self.dims), L.i32_array(self.Ks)
        self.w_arr, self.b_arr, self.c_arr = L.ptr_array(self.ws), L.ptr_array(self.bs), L.ptr_array(self.cbs)
        self.device = self.ws[0].device
        self.dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._ws_bytes = {}
        # the fused encoder's packed weight image (frozen weights only, see packed_ptr)
        nf = L.lib().gr_rq_encoder_pack_floats(len(self.ws), self.dims_c)
        self.packed = torch.empty(nf, dtype=torch.float32, device=self.device) if nf else None
        self._pack_key = None

    # Re-use one packed encoder image across calls, re-packed whenever a weight's version counter
    # (load_state_dict, optimizer steps, any in-place op) or the graph-replay epoch moves (a
    # replayed training graph updates the weights without a version bump: ops.weights_changed).
    # A write that bypasses both (``param.data[...] = ...``) must call weights_changed(), or the
    # owner runs with ``RQVAE.freeze_encoder(False)``: every call then packs the current weights
    # into its workspace (one extra launch, 4 us per C2 call, profiles/r04/ab_rq_pack.txt).
    frozen = True

    def packed_ptr(self):
        """Device pointer of the up-to-date packed encoder image; None: pack per call
        (``frozen = False``, or not the fused encoder shape)."""
        if self.packed is None or not self.frozen:
            return None
        key = tuple(w._version for w in self.ws) + (_WEIGHT_EPOCH[0],)
        capturing = torch.cuda.is_current_stream_capturing()
        if key != self._pack_key and capturing:
            # a pack recorded into a graph would run only at replay, leaving the eager image stale
            raise RuntimeError("rq_encode: the packed encoder image is out of date inside a graph capture; "
                               "run one eager get_indices after the last weight change, then capture "
                               "(graphs that encode must be re-captured after weight changes)")
        if capturing:
            # a captured graph bakes in this image's pointer: keep the image alive for the binding's
            # lifetime, so replays after a later re-pack read the old weights, never freed memory
            refs = self.__dict__.setdefault("_graph_images", [])
            if not any(r is self.packed for r in refs):
                refs.append(self.packed)
        if key != self._pack_key:
            if self._pack_key is not None:
                # a re-pack writes a fresh image on this stream; the previous one goes back to the
                # caching allocator, which does not hand it out again before the work of every
                # stream recorded on it (below) has finished
                self.packed = torch.empty_like(self.packed)
                self._streams = set()
            with L.on(self.device):
                L.check(L.lib().gr_rq_encoder_pack_f32(len(self.ws), self.dims_c, self.w_arr, L.ptr(self.packed),
                                                       L.stream_of(self.device)), "gr_rq_encoder_pack_f32")
            self._pack_key = key
        st = L.stream_of(self.device)
        streams = getattr(self, "_streams", None)
        if streams is None:
            streams = self._streams = set()
        if st not in streams:   # an encode on another stream than the allocating one
            self.packed.record_stream(torch.cuda.current_stream(self.device))
            streams.add(st)
        return self.packed.data_ptr()

    def encode_fast(self, x):
        """rq_encode's common call -- fp32 contiguous [n, in_dim] rows on the binding's (current)
        device, eager, semantic IDs only -- with the per-call host work cut to the checks and the
        launch (the reference's get_indices(x[64]) is host-bound).  None: not that case; the
        general path (which also raises the errors) runs instead.  Same C call, same results."""
        if (x.dtype is not torch.float32 or x.dim() != 2 or x.shape[1] != self.in_dim or not x.is_cuda
                or not x.is_contiguous() or x.get_device() != self.dev_index
                or self.dev_index != torch.cuda.current_device() or torch.cuda.is_current_stream_capturing()):
            return None
        pk = self.packed_ptr()
        n = x.shape[0]
        st = L.stream_of(self.device)
        nbytes = self._ws_bytes.get(n) or self.workspace_bytes(n)
        ws = _SCRATCH.get((self.dev_index, st))
        if ws is None or ws.numel() < nbytes:
            ws = scratch(nbytes, self.device)
        idx = torch.empty((n, len(self.cbs)), dtype=torch.int64, device=self.device)
        rc = L.lib().gr_rq_encode_packed_f32(x.data_ptr(), n, self.n_linear, self.dims_c, self.w_arr, self.b_arr,
                                             pk, len(self.cbs), self.ks_c, self.c_arr, idx.data_ptr(), None, None,
                                             None, ws.data_ptr(), nbytes, st)
        if rc:
            L.check(rc, "gr_rq_encode_packed_f32")
        return idx

    def workspace_bytes(self, n):
        nb = self._ws_bytes.get(n)
        if nb is None:
            nb = L.lib().gr_rq_encode_workspace_bytes(n, len(self.ws), self.dims_c, len(self.cbs), self.ks_c)
            if nb == 0:
                raise RuntimeError("rq_encode: bad encoder description")
            if len(self._ws_bytes) < 64:
                self._ws_bytes[n] = nb
        return nb


# Bumped by every replay of a captured training step (its optimizer updates parameters in place
# without touching their version counters), so cached weight images re-pack after it.
_WEIGHT_EPOCH = [0]


def weights_changed():
    """Tell the cached kernel bindings that parameters changed behind torch's version counters."""
    _WEIGHT_EPOCH[0] += 1


def mkl_plan(m, k, n):
    """MKL's accumulation order for one reference CPU sgemm call of ``m`` rows, inner size ``k``,
    ``n`` outputs (``gr_mkl_plan``): (kind, block width, pinned), kind in chain / gemv16 / small16."""
    kind, kb = ctypes.c_int32(0), ctypes.c_int32(0)
    pinned = L.lib().gr_mkl_plan(int(m), int(k), int(n), ctypes.byref(kind), ctypes.byref(kb))
    return ("chain", "gemv16", "small16")[kind.value], kb.value, bool(pinned)


def rq_binding(owner, weights_fn):
    """Cached :class:`RqBinding` on ``owner`` (an RQVAE): rebuilt when any parameter's storage moved
    (``.to()``, ``param.data = ...``); in-place updates (``load_state_dict``, optimiser steps) are
    seen through the same pointers.  ``weights_fn() -> (weights, biases, codebooks)``, the LIVE
    parameters (not detached copies: their pointers are the cache key)."""
    c = owner.__dict__.get("_gr_rq_binding")
    if c is not None:
        tensors, key, b = c
        if b.direct and tuple(t.data_ptr() for t in tensors) == key:
            return b
    ws, bs, cbs = weights_fn()
    tensors = list(ws) + list(bs) + list(cbs)
    b = RqBinding(ws, bs, cbs)
    owner.__dict__["_gr_rq_binding"] = (tensors, tuple(t.data_ptr() for t in tensors), b)
    return b


def rq_encode(x, weights=None, biases=None, codebooks=None, with_gap=False, with_z=False, binding=None):
    """RQVAE.get_indices(xs, use_sk=False): encoder MLP + residual quantization (rqvae.py:67-71).

    Returns ``idx`` [n, L] int64, plus ``best`` and ``gap`` [n, L] (best distance and second-best
    minus best) and the encoder output ``z`` when requested.  ``binding`` (an :class:`RqBinding`)
    replaces ``weights`` / ``biases`` / ``codebooks``.
    """
    if binding is not None and not with_gap and not with_z:
        idx = binding.encode_fast(x)
        if idx is not None:
            return idx
    b = binding if binding is not None else RqBinding(weights, biases, codebooks)
    L.require_gpu(x)
    x2 = L.as_f32(x)
    if x2.dim() != 2 or x2.shape[1] != b.in_dim:
        raise RuntimeError(f"rq_encode: expected [n, {b.in_dim}] inputs, got {tuple(x2.shape)}")
    dev = x2.device
    if dev != b.device:
        raise RuntimeError(f"rq_encode: inputs on {dev}, parameters on {b.device}")
    n = x2.shape[0]
    nbytes = b.workspace_bytes(n)
    wsp = scratch(nbytes, dev)
    nl = len(b.cbs)
    idx = torch.empty((n, nl), dtype=torch.int64, device=dev)
    gap = torch.empty((n, nl), dtype=torch.float32, device=dev) if with_gap else None
    best = torch.empty((n, nl), dtype=torch.float32, device=dev) if with_gap else None
    z = torch.empty((n, b.dims[-1]), dtype=torch.float32, device=dev) if with_z else None
    with L.on(dev):
        L.check(L.lib().gr_rq_encode_packed_f32(x2.data_ptr(), n, b.n_linear, b.dims_c, b.w_arr, b.b_arr,
                                                b.packed_ptr(), nl, b.ks_c, b.c_arr, idx.data_ptr(), L.ptr(best),
                                                L.ptr(gap), L.ptr(z), wsp.data_ptr(), nbytes, L.stream_of(dev)),
                "gr_rq_encode_packed_f32")
    out = [idx]
    if with_gap:
        out += [best, gap]
    if with_z:
        out.append(z)
    return out[0] if len(out) == 1 else tuple(out)


_EXACT_ACTS = {"relu": 1, "none": 0, None: 0, "leakyrelu": 4}


def rq_mlp(x, weights, biases, bn=None, act="relu", group_sizes=None):
    """MLPLayers.forward (RQ-VAE/models/layers.py:18-43, eval): the encoder output ``z`` alone, in
    the reference's CPU order bit for bit (``gr_mlp_exact_f32``: the fused kernel for in -> 256 ->
    128 -> 32 ReLU MLPs, exact layer-wise launches otherwise, the per-row kernel for 1-15-row
    calls).  ``bn``: None, or (means, vars, weights, biases, eps) of the eval BatchNorm1d after every
    Linear but the last (weights / biases entries may be None: affine off); ``act``: relu /
    leakyrelu / none.  ``group_sizes``: consecutive row groups, each ONE reference call (MKL's order
    depends on the call's row count; ``gr_mlp_exact_groups_f32``)."""
    L.require_gpu(x, *weights)
    x2 = L.as_f32(x)
    n = x2.shape[0]
    ws = [L.as_f32(w) for w in weights]
    bs = [L.as_f32(b) for b in biases] if biases is not None else None
    dims = [x2.shape[1]] + [w.shape[0] for w in ws]
    for i, w in enumerate(ws):
        if w.shape[1] != dims[i]:
            raise RuntimeError(f"rq_mlp: Linear {i} expects {w.shape[1]} inputs, got {dims[i]}")
    if act not in _EXACT_ACTS:
        raise RuntimeError(f"rq_mlp: activation {act} has no exact kernel (relu / leakyrelu / none)")
    dev = x.device
    lib = L.lib()
    dims_c = L.i32_array(dims)
    nbytes = lib.gr_rq_mlp_workspace_bytes(n, len(ws), dims_c)
    wsp = L.workspace(nbytes, dev)
    z = torch.empty((n, dims[-1]), dtype=torch.float32, device=dev)
    bn_arrs = [None] * 4
    eps = 0.0
    keep = []
    if bn is not None:
        means, vars_, bws, bbs, eps = bn
        for j, group in enumerate((means, vars_, bws, bbs)):
            if group is None or all(t is None for t in group):
                continue
            ts = [L.as_f32(t) for t in group]
            keep.append(ts)
            bn_arrs[j] = L.ptr_array(ts)
    with L.on(dev):
        if group_sizes is not None:
            sizes = [int(g) for g in group_sizes]
            if sum(sizes) != n or any(g < 1 for g in sizes):
                raise RuntimeError("rq_mlp: group sizes must be positive and sum to the batch")
            # Groups MKL runs as k-block chains (>= 16 rows) whose per-layer blocks match those of ONE
            # call over all of them produce the same bits in that call: they go through the MFMA
            # kernels together; the rest (1-15-row orders) through the per-row kernel, group by group.
            plans = {}

            def plan(m):
                if m not in plans:
                    plans[m] = tuple(mkl_plan(m, dims[i], dims[i + 1])[:2] for i in range(len(ws)))
                return plans[m]

            big = [i for i, g in enumerate(sizes) if all(k == "chain" for k, _ in plan(g))]
            while big:   # the kept groups' one call must have every kept group's own order
                pb = plan(sum(sizes[i] for i in big))
                keep = [i for i in big if plan(sizes[i]) == pb]
                if keep == big:
                    break
                big = keep
            small = [i for i in range(len(sizes)) if i not in set(big)]
            offs = [0]
            for g in sizes:
                offs.append(offs[-1] + g)

            def rows_of(sel):
                return torch.cat([torch.arange(offs[i], offs[i + 1], device=dev) for i in sel])

            if small:
                rs = rows_of(small) if big else None
                xs = x2 if rs is None else x2.index_select(0, rs).contiguous()
                zs = z if rs is None else torch.empty((xs.shape[0], dims[-1]), dtype=torch.float32, device=dev)
                ptr = _group_ptr([sizes[i] for i in small], dev)
                L.check(lib.gr_mlp_exact_groups_f32(L.ptr(xs), xs.shape[0], len(ws), dims_c, L.ptr_array(ws),
                                                    L.ptr_array(bs) if bs is not None else None, *bn_arrs,
                                                    float(eps), _EXACT_ACTS[act], L.ptr(ptr), len(small),
                                                    L.ptr(zs), L.stream_of(dev)), "gr_mlp_exact_groups_f32")
                if rs is not None:
                    z.index_copy_(0, rs, zs)
            if big:
                rb = rows_of(big) if small else None
                xb = x2 if rb is None else x2.index_select(0, rb).contiguous()
                nb2 = xb.shape[0]
                zb = z if rb is None else torch.empty((nb2, dims[-1]), dtype=torch.float32, device=dev)
                nbytes2 = lib.gr_rq_mlp_workspace_bytes(nb2, len(ws), dims_c)
                wsp2 = L.workspace(nbytes2, dev)
                L.check(lib.gr_mlp_exact_f32(L.ptr(xb), nb2, len(ws), dims_c, L.ptr_array(ws),
                                             L.ptr_array(bs) if bs is not None else None, *bn_arrs, float(eps),
                                             _EXACT_ACTS[act], L.ptr(zb), L.ptr(wsp2), nbytes2, L.stream_of(dev)),
                        "gr_mlp_exact_f32")
                if rb is not None:
                    z.index_copy_(0, rb, zb)
            return z
        L.check(lib.gr_mlp_exact_f32(L.ptr(x2), n, len(ws), dims_c, L.ptr_array(ws),
                                     L.ptr_array(bs) if bs is not None else None, *bn_arrs, float(eps),
                                     _EXACT_ACTS[act], L.ptr(z), L.ptr(wsp), nbytes, L.stream_of(dev)),
                "gr_mlp_exact_f32")
    return z


def rq_encode_sk(x, weights, biases, codebooks, sk_eps, sk_iters, group_sizes=None):
    """RQVAE.get_indices(xs, use_sk=True) (RQ-VAE/models/rqvae.py:67-71 with vq.py:76-84) for
    independent row groups in ONE launch: ``group_sizes`` partitions the rows of ``x`` into
    consecutive groups, each one reference call (default: the whole batch is one group)."""
    L.require_gpu(x, *weights, *codebooks)
    return rq_quantize_sk(rq_mlp(x, weights, biases, group_sizes=group_sizes), codebooks, sk_eps, sk_iters,
                          group_sizes)


def rq_encode_z(z, codebooks, with_gap=False):
    """``get_indices`` from encoder outputs computed elsewhere (e.g. a BatchNorm encoder)."""
    return rq_quantize(z, codebooks, with_gap=with_gap)


_GROUP_PTRS = {}


def _group_ptr(sizes, dev):
    """Device copy of the group offsets [0, s0, s0+s1, ...].  The one-group form (a training batch)
    is cached per (n, device) and never freed, so a captured training step (RqTrainGraph) replays
    the Sinkhorn launch with no host-to-device copy and a pointer that stays valid."""
    if len(sizes) != 1:
        return torch.tensor([0] + list(itertools.accumulate(sizes)), dtype=torch.int64).to(dev)
    key = (sizes[0], str(dev))
    t = _GROUP_PTRS.get(key)
    if t is None:
        t = torch.tensor([0, sizes[0]], dtype=torch.int64).to(dev)
        _GROUP_PTRS[key] = t
    return t


def rq_quantize_sk(z, codebooks, sk_eps, sk_iters, group_sizes=None):
    """ResidualVectorQuantizer.forward(z, use_sk=True) indices (rq.py:39-56, vq.py:63-84): per level,
    Sinkhorn over the group's distances where ``sk_eps[l] > 0``, plain argmin otherwise."""
    L.require_gpu(z, *codebooks)
    z = L.as_f32(z)
    n = z.shape[0]
    cbs = [L.as_f32(c) for c in codebooks]
    e = z.shape[1]
    Ks = [c.shape[0] for c in cbs]
    sizes = [n] if group_sizes is None else [int(s) for s in group_sizes]
    if sum(sizes) != n or any(s < 1 for s in sizes):
        raise RuntimeError("rq_encode_sk: group sizes must be positive and sum to the batch")
    dev = z.device
    ptr = _group_ptr(sizes, dev)
    lib = L.lib()
    ks_c = L.i32_array(Ks)
    eps_c = (ctypes.c_double * len(cbs))(*[float(v) for v in sk_eps])
    nbytes = lib.gr_rq_encode_sk_workspace_bytes(n, e, len(cbs), ks_c)
    wsp = L.workspace(nbytes, dev)
    idx = torch.empty((n, len(cbs)), dtype=torch.int64, device=dev)
    with L.on(dev):
        L.check(lib.gr_rq_encode_sk_f32(L.ptr(z), n, e, len(cbs), ks_c, L.ptr_array(cbs), eps_c,
                                        int(sk_iters), L.ptr(ptr), len(sizes), L.ptr(idx), L.ptr(wsp),
                                        nbytes, L.stream_of(dev)), "gr_rq_encode_sk_f32")
    return idx


class SasrecBinding:
    """Device-pointer view of a SASRec module's parameters (``gr_sasrec_params``).

    Built once per parameter set and cached on the module (:func:`sasrec_binding`); the pointers
    are the parameters' own storage, so in-place weight updates and ``load_state_dict`` are seen.
    """

    def __init__(self, model):
        self.keep = []
        self.direct = True           # every pointer is the parameter's own storage (no copies)
        f = self._f
        nb = model.num_blocks
        p = L.SasrecParams()
        p.d, p.n_blocks, p.n_heads, p.mlp = model.d, nb, model.num_heads, model.mlp_layer
        p.max_len = model.pos_emb.weight.shape[0]
        p.eps = float(model.layernorm_eps)
        p.item_rows = model.item_emb.weight.shape[0]
        p.item_emb = f(model.item_emb.weight)
        p.pos_emb = f(model.pos_emb.weight)
        arr = self._arr
        p.attn_ln_w = arr([m.weight for m in model.attention_layernorms])
        p.attn_ln_b = arr([m.bias for m in model.attention_layernorms])
        p.in_proj_w = arr([m.in_proj_weight for m in model.attention_layers])
        p.in_proj_b = arr([m.in_proj_bias for m in model.attention_layers])
        p.out_proj_w = arr([m.out_proj.weight for m in model.attention_layers])
        p.out_proj_b = arr([m.out_proj.bias for m in model.attention_layers])
        p.ffn_ln_w = arr([m.weight for m in model.forward_layernorms])
        p.ffn_ln_b = arr([m.bias for m in model.forward_layernorms])
        p.ffn1_w = arr([m[0].weight for m in model.forward_layers])
        p.ffn1_b = arr([m[0].bias for m in model.forward_layers])
        p.ffn2_w = arr([m[3].weight for m in model.forward_layers])
        p.ffn2_b = arr([m[3].bias for m in model.forward_layers])
        p.last_ln_w = f(model.last_layernorm.weight)
        p.last_ln_b = f(model.last_layernorm.bias)
        self.p = p
        self.p_ref = ctypes.byref(p)
        self.device = model.item_emb.weight.device
        self._ws = {}

    def _f(self, t):
        L.require_gpu(t)
        t2 = L.as_f32(t.detach())
        self.direct &= t2.data_ptr() == t.data_ptr()
        self.keep.append(t2)
        return t2.data_ptr()

    def _arr(self, ts):
        a = (ctypes.c_void_p * max(1, len(ts)))(*[self._f(t) for t in ts])
        self.keep.append(a)
        return ctypes.cast(a, ctypes.c_void_p)

    def workspace_bytes(self, B, n):
        key = (0, B, n)
        nb = self._ws.get(key)
        if nb is None:
            nb = L.lib().gr_sasrec_workspace_bytes(self.p_ref, B, n)
            if len(self._ws) < 256:
                self._ws[key] = nb
        return nb

    def rank_workspace_bytes(self, B, n):
        key = (1, B, n)
        nb = self._ws.get(key)
        if nb is None:
            nb = (L.lib().gr_sasrec_rank_workspace_bytes(self.p_ref, B, n),
                  L.lib().gr_score_count_workspace_bytes(B))
            if len(self._ws) < 256:
                self._ws[key] = nb
        return nb


def sasrec_binding(model):
    """Cached :class:`SasrecBinding` of ``model``: reused while every parameter's storage pointer
    is unchanged (checked per call, ~5 us for SASRec's 34 tensors); rebuilt after ``.to()`` or a
    ``param.data = ...`` swap, and on every call when a parameter is not contiguous fp32 (then the
    binding holds copies).  This is what makes a ``predict`` at the reference's eval batch of 128
    (SASRec/evaluate.py:13, 26) cost one launch on the host."""
    c = model.__dict__.get("_gr_sas_binding")
    if c is not None:
        params, key, b = c
        if b.direct and tuple(q.data_ptr() for q in params) == key:
            return b
    params = list(model.parameters())
    b = SasrecBinding(model)
    model.__dict__["_gr_sas_binding"] = (params, tuple(q.data_ptr() for q in params), b)
    return b


def _sas_ids(log_seqs, binding):
    L.require_gpu(log_seqs)
    if log_seqs.dim() != 2:
        raise RuntimeError("SASRec expects log_seqs of shape [B, n]")
    if log_seqs.device != binding.device:
        raise RuntimeError(f"log_seqs on {log_seqs.device}, model on {binding.device}")
    return log_seqs.to(torch.int64).contiguous()


def _check_err(err):
    if CHECK:
        check_errors(err.device)


def sasrec_forward(binding, log_seqs, last_only=False):
    ids = _sas_ids(log_seqs, binding)
    B, n = ids.shape
    dev = ids.device
    d = binding.p.d
    out = torch.empty((B, d) if last_only else (B, n, d), dtype=torch.float32, device=dev)
    nbytes = binding.workspace_bytes(B, n)
    wsp = scratch(nbytes, dev)
    err = err_flag(dev)
    with L.on(dev):
        L.check(L.lib().gr_sasrec_forward_f32(binding.p_ref, L.ptr(ids), B, n, L.ptr(out),
                                              1 if last_only else 0, L.ptr(wsp), nbytes, L.ptr(err),
                                              L.stream_of(dev)), "gr_sasrec_forward_f32")
    _check_err(err)
    return out


def sasrec_rank(binding, log_seqs, targets, mask_col0=True):
    """One batch of SASRec/evaluate.py:26-32 in ONE C-ABI call (``gr_sasrec_rank_f32``): the 1-based
    strict rank of each target over the full catalog, column 0 taken as -1e9 when ``mask_col0``,
    from the forward's last hidden states -- the logits are never written.  Bitwise the ranks of
    ``ops.rank(predict(seqs), targets)`` (the same fp32 scoring chain)."""
    ids = _sas_ids(log_seqs, binding)
    B, n = ids.shape
    t = targets.reshape(-1)
    if t.dtype != torch.int64:
        t = t.to(torch.int64)
    if not t.is_contiguous():
        t = t.contiguous()
    if t.shape[0] != B:
        raise RuntimeError(f"sasrec_rank: {t.shape[0]} targets for {B} sequences")
    dev = ids.device
    nbytes, cnb = binding.rank_workspace_bytes(B, n)
    wsp = scratch(nbytes, dev)
    out = torch.empty(B, dtype=torch.int64, device=dev)
    err = err_flag(dev)
    cws, key = _count_workspace(dev, cnb)
    with L.on(dev):
        try:
            L.check(L.lib().gr_sasrec_rank_f32(binding.p_ref, ids.data_ptr(), B, n, t.data_ptr(),
                                               1 if mask_col0 else 0, out.data_ptr(), wsp.data_ptr(), nbytes,
                                               L.ptr(cws), cnb, err.data_ptr(),
                                               L.stream_of(dev)), "gr_sasrec_rank_f32")
        except Exception:
            if key is not None:
                _COUNT_WS.pop(key, None)
            raise
    _check_err(err)
    return out


LOGITS_ROW_ALIGN = 32  # floats: one 128-byte line


def logits_buffer(B, rows, device):
    """A fresh ``[B, rows]`` fp32 logits tensor whose rows are ``rows`` rounded up to 32 floats apart
    (a view of a ``[B, ld]`` allocation), so every row starts on a 128-byte line and the scoring
    kernel stores whole lines straight from its accumulators.  The reference's callers
    (evaluate.py:27-32, train.py:45-48: in-place ``[:, 0]`` mask, ``gather``, ``>`` + ``sum``) work on
    it unchanged; ``.contiguous()`` gives a packed copy."""
    ld = -(-rows // LOGITS_ROW_ALIGN) * LOGITS_ROW_ALIGN
    return torch.empty((B, ld), dtype=torch.float32, device=device)[:, :rows]


def sasrec_predict(binding, log_seqs, out=None):
    """model.py:98-108 through ``gr_sasrec_predict_ld_f32``.  ``out`` (optional) may be any
    ``[B, item_rows]`` fp32 tensor with unit column stride; by default a row-padded
    :func:`logits_buffer` is returned."""
    ids = _sas_ids(log_seqs, binding)
    B, n = ids.shape
    dev = ids.device
    rows = binding.p.item_rows
    logits = out if out is not None else logits_buffer(B, rows, dev)
    if (logits.shape != (B, rows) or logits.dtype != torch.float32 or logits.device != dev
            or (B > 1 and logits.stride(1) != 1) or logits.stride(0) < rows):
        raise ValueError("sasrec_predict: out must be fp32 [B, item_rows] on the ids' device with unit column stride")
    ld = logits.stride(0) if B > 1 else rows
    nbytes = binding.workspace_bytes(B, n)
    wsp = scratch(nbytes, dev)
    err = err_flag(dev)
    with L.on(dev):
        L.check(L.lib().gr_sasrec_predict_ld_f32(binding.p_ref, L.ptr(ids), B, n,
                                                 L.ptr(logits), ld, L.ptr(wsp), nbytes, L.ptr(err),
                                                 L.stream_of(dev)), "gr_sasrec_predict_ld_f32")
    _check_err(err)
    return logits


# --------------------------------------------------------------------------------------------
# Training-side scoring (SASRec/train.py:131-160)

class _SampledBCE(torch.autograd.Function):
    """``(batch_loss, batch_valid_t)`` of train.py:134-158 with the score matrix never formed;
    differentiable in ``feats`` and ``table`` (gr_sampled_bce_fwd_f32 / gr_sampled_bce_bwd_f32)."""

    @staticmethod
    def forward(ctx, feats, table, targets, negs, eps):
        B, n, d = feats.shape
        rows = table.shape[0]
        J = negs.shape[1]
        dev = feats.device
        row_loss = torch.empty(B * n, dtype=torch.float32, device=dev)
        coef = torch.empty(B * n * (J + 1), dtype=torch.float32, device=dev)
        sums = torch.empty(2, dtype=torch.float32, device=dev)
        err = err_flag(dev)
        with L.on(dev):
            L.check(L.lib().gr_sampled_bce_fwd_f32(L.ptr(feats), B, n, d, L.ptr(table), rows,
                                                   L.ptr(targets), L.ptr(negs), J, float(eps),
                                                   L.ptr(row_loss), L.ptr(coef), L.ptr(sums),
                                                   L.ptr(err), L.stream_of(dev)),
                    "gr_sampled_bce_fwd_f32")
        _check_err(err)
        ctx.save_for_backward(feats, table, targets, negs, coef)
        valid = sums[1]
        ctx.mark_non_differentiable(valid)
        return sums[0], valid

    @staticmethod
    def backward(ctx, g_loss, g_valid):
        feats, table, targets, negs, coef = ctx.saved_tensors
        B, n, d = feats.shape
        rows = table.shape[0]
        dev = feats.device
        g = g_loss.to(device=dev, dtype=torch.float32).reshape(1).contiguous()
        dfeats = torch.empty_like(feats)
        dtable = torch.empty_like(table)
        with L.on(dev):
            L.check(L.lib().gr_sampled_bce_bwd_f32(L.ptr(feats), B, n, d, L.ptr(table), rows,
                                                   L.ptr(targets), L.ptr(negs), negs.shape[1],
                                                   L.ptr(coef), L.ptr(g), L.ptr(dfeats),
                                                   L.ptr(dtable), L.stream_of(dev)),
                    "gr_sampled_bce_bwd_f32")
        return dfeats, dtable, None, None, None


def sampled_bce_loss(seq_features, item_emb_weight, target_o_t, neg_samples, eps):
    """train.py:134-158 in one fused op: returns ``(batch_loss, batch_valid_t)`` as device scalars,
    equal to the reference's ``(pos_loss + neg_loss).sum()`` and ``mask.sum()`` over the
    ``[B, n, item_num+1]`` score matrix it forms (this op never forms it).  ``batch_loss`` is
    differentiable in ``seq_features`` [B, n, d] and ``item_emb_weight`` [item_num+1, d]; the caller
    divides by ``batch_valid_t`` (train.py:161-164) and calls ``backward()`` as before."""
    L.require_gpu(seq_features, item_emb_weight, target_o_t, neg_samples)
    if seq_features.dim() != 3 or item_emb_weight.dim() != 2 or seq_features.shape[2] != item_emb_weight.shape[1]:
        raise RuntimeError("sampled_bce_loss: seq_features [B, n, d] and item_emb_weight [rows, d] expected")
    B, n, _ = seq_features.shape
    if tuple(target_o_t.shape) != (B, n) or neg_samples.dim() != 2 or neg_samples.shape[0] != B:
        raise RuntimeError("sampled_bce_loss: target_o_t [B, n] and neg_samples [B, num_neg] expected")
    return _SampledBCE.apply(L.as_f32(seq_features), L.as_f32(item_emb_weight),
                             target_o_t.to(torch.int64).contiguous(),
                             neg_samples.to(torch.int64).contiguous(), eps)


_NEG_CALLS = itertools.count()


def neg_samples(seq, item_num, num_neg=1, seed=None, seed_tensor=None):
    """train.py:15-30 ``get_neg_samples(seq, item_num, num_neg)`` on the GPU: ``[B, num_neg]`` int64,
    per row distinct items uniform over ``[1, item_num]`` minus the row's non-zero history (the
    reference's distribution; not numpy's random stream).  ``seed`` defaults to a fresh value per
    call drawn from torch's global generator, so ``torch.manual_seed`` makes runs repeatable.

    A row whose population (``item_num`` minus its distinct history) is smaller than ``num_neg``
    raises ValueError, as numpy's ``choice(replace=False)`` does.  That can only happen when
    ``n + num_neg > item_num`` (the history holds at most ``n`` distinct items), and only then does
    this call synchronise to check; otherwise every candidate is accepted with probability
    >= 1/2 and the kernel's 4096 rounds of 64 draws cannot fall short.  Unfilled rows hold -1.

    ``seed_tensor`` (a CUDA int64 tensor of one element): the stream is keyed by ``seed ^
    seed_tensor`` read on the device, and ``seed_tensor`` is advanced by one on the stream after
    the draw -- the form a captured graph replays with fresh negatives (``SasTrainStepGraph``)."""
    L.require_gpu(seq)
    s = seq.to(torch.int64).contiguous()
    if s.dim() != 2:
        raise RuntimeError("neg_samples: seq must be [B, n]")
    B, n = s.shape
    if seed is None:
        seed = 0 if seed_tensor is not None else int(torch.randint(0, 2 ** 62, (1,)).item()) ^ next(_NEG_CALLS)
    out = torch.empty((B, num_neg), dtype=torch.int64, device=s.device)
    err = err_flag(s.device)
    with L.on(s.device):
        if seed_tensor is not None:
            if seed_tensor.dtype != torch.int64 or seed_tensor.numel() != 1 or seed_tensor.device != s.device:
                raise RuntimeError("neg_samples: seed_tensor must be one int64 element on the sequences' device")
            L.check(L.lib().gr_neg_samples_dseed(L.ptr(s), B, n, int(item_num), int(num_neg),
                                                 int(seed) & (2 ** 64 - 1), L.ptr(seed_tensor), L.ptr(out),
                                                 L.ptr(err), L.stream_of(s.device)), "gr_neg_samples_dseed")
            seed_tensor.add_(1)
        else:
            L.check(L.lib().gr_neg_samples(L.ptr(s), B, n, int(item_num), int(num_neg), int(seed) & (2 ** 64 - 1),
                                           L.ptr(out), L.ptr(err), L.stream_of(s.device)), "gr_neg_samples")
    # a short population is possible only when 2 (n + num_neg) > item_num; never synchronise inside a
    # graph capture (the captured step classes check once per replay instead)
    if (CHECK or 2 * (n + num_neg) > item_num) and not torch.cuda.is_current_stream_capturing():
        check_errors(s.device)
    return out


# --------------------------------------------------------------------------------------------
# Transformer training forward / backward (SASRec/model.py:49-96 under train.py:131 and :161-172)

_DROP_SEED = {}


def dropout_seed(device):
    """The device's dropout seed word: every train-mode forward snapshots it and advances it by one
    on the stream (a captured step therefore replays with fresh masks).  Initialised from torch's
    global generator, so ``torch.manual_seed`` makes runs repeatable."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    t = _DROP_SEED.get(idx)
    if t is None:
        t = torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).to(torch.device("cuda", idx))
        _DROP_SEED[idx] = t
    return t


def sasrec_train_supported(model, n):
    return (n <= 64 and n <= model.pos_emb.weight.shape[0] and model.d <= 64
            and model.d % model.num_heads == 0 and model.mlp_layer <= 128 and 1 <= model.num_blocks <= 8)


def _train_params(model):
    """The parameters the transformer's forward reads, in the order _SasTrain returns gradients."""
    ps = [model.item_emb.weight, model.pos_emb.weight]
    for la, at, lf, ff in zip(model.attention_layernorms, model.attention_layers, model.forward_layernorms,
                              model.forward_layers):
        ps += [la.weight, la.bias, at.in_proj_weight, at.in_proj_bias, at.out_proj.weight, at.out_proj.bias,
               lf.weight, lf.bias, ff[0].weight, ff[0].bias, ff[3].weight, ff[3].bias]
    return ps + [model.last_layernorm.weight, model.last_layernorm.bias]


class _SasTrain(torch.autograd.Function):
    """Train-mode SASRec forward (dropout on) and its backward on the kernels of sasrec_train.hip:
    one launch each.  The backward leaves every parameter gradient but the item table's as a
    per-sequence partial row of one [B, V] buffer (dW = dG^T A over the sequence's rows, bias and
    LayerNorm column sums, positional rows), summed over B here; item-table rows are scattered in
    the kernel."""

    @staticmethod
    def forward(ctx, seqs, binding, p_drop, seed_snap, *params):
        B, n = seqs.shape
        p = binding.p
        d, m, nb, H = p.d, p.mlp, p.n_blocks, p.n_heads
        dev = seqs.device
        R = B * n
        e = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)   # noqa: E731
        bufs = {"xin": e(nb, R, d), "hs": e(nb, R, d), "qkv": e(nb, R, 3 * d), "prob": e(nb, B, H, n, n),
                "os": e(nb, R, d), "x1": e(nb, R, d), "fs": e(nb, R, d), "zs": e(nb, R, m), "us": e(nb, R, m),
                "xl": e(R, d)}
        out = e(B, n, d)
        err = err_flag(dev)
        cb = L.SasrecTrainBufs(**{k: v.data_ptr() for k, v in bufs.items()})
        with L.on(dev):
            L.check(L.lib().gr_sasrec_train_fwd_f32(ctypes.byref(p), L.ptr(seqs), B, n, float(p_drop), 0,
                                                    L.ptr(seed_snap), ctypes.byref(cb), L.ptr(out), L.ptr(err),
                                                    L.stream_of(dev)), "gr_sasrec_train_fwd_f32")
        _check_err(err)
        ctx.binding, ctx.p_drop, ctx.bufs, ctx.seqs, ctx.seed = binding, p_drop, bufs, seqs, seed_snap
        ctx.shapes = (B, n, d, m, nb, params[1].shape[0])
        return out

    @staticmethod
    def backward(ctx, dout):
        B, n, d, m, nb, max_len = ctx.shapes
        bufs, seqs = ctx.bufs, ctx.seqs
        dev = seqs.device
        p = ctx.binding.p
        vw = L.lib().gr_sasrec_train_vec_width(ctypes.byref(p), n)
        g_vec = torch.empty((B, vw), dtype=torch.float32, device=dev)
        g_item = torch.zeros((p.item_rows, d), dtype=torch.float32, device=dev)
        cb = L.SasrecTrainBufs(g_vec=g_vec.data_ptr(), **{k: v.data_ptr() for k, v in bufs.items()})
        dout = dout.contiguous().float()
        with L.on(dev):
            L.check(L.lib().gr_sasrec_train_bwd_f32(ctypes.byref(p), L.ptr(seqs), B, n, float(ctx.p_drop), 0,
                                                    L.ptr(ctx.seed), ctypes.byref(cb), L.ptr(dout), L.ptr(g_item),
                                                    L.stream_of(dev)), "gr_sasrec_train_bwd_f32")
        vec = g_vec.sum(0)   # every parameter's gradient but the item table's, in parameter order
        shapes = [(d,), (d,), (3 * d, d), (3 * d,), (d, d), (d,), (d,), (d,), (m, d), (m,), (d, m), (d,)] * nb
        shapes += [(d,), (d,)]
        grads, off = [], 0
        for shp in shapes:
            k = 1
            for x in shp:
                k *= x
            grads.append(vec[off:off + k].view(shp))
            off += k
        # rows n.. of pos_emb get zeros (a pad kernel rather than a copy into a zeros tensor, which
        # keeps memset / memcpy nodes out of a captured step's graph)
        dpos = torch.nn.functional.pad(vec[off:off + n * d].view(n, d), (0, 0, 0, max_len - n))
        return (None, None, None, None, g_item, dpos, *grads)


def sasrec_train_forward(model, log_seqs):
    """``model.forward(log_seqs)`` in train mode with grad (SASRec/train.py:131): the transformer
    forward with dropout on the kernels, differentiable in every parameter it reads."""
    seqs = log_seqs.to(torch.int64).contiguous()
    L.require_gpu(seqs)
    seed = dropout_seed(seqs.device)
    snap = seed + 0              # this step's masks (forward and backward read the same word); a kernel, not a copy
    seed.add_(1)
    return _SasTrain.apply(seqs, sasrec_binding(model), float(model.dropout), snap, *_train_params(model))


class SasTrainStepGraph:
    """The training-side scoring step of SASRec/train.py:131-167 -- negatives (train.py:142),
    scores + sampled BCE (134-158), ``loss = batch_loss / batch_valid_t`` (161-164) and its backward
    into ``feats.grad`` / ``table.grad`` -- captured once as a graph (hipGraph via
    ``torch.cuda.graph``) and replayed: one launch per step instead of ~20 host-issued ones.

    ``feats`` [B, n, d] and ``table`` [rows, d] are leaf tensors with ``requires_grad``; ``inputs``
    (the sequences the negatives avoid) and ``targets`` are the step's static inputs: copy a new
    batch into them before ``replay()``.  Each replay draws fresh negatives (device-side seed).
    ``replay()`` returns the static ``(batch_loss, batch_valid_t)`` device scalars and leaves the
    gradients in ``.grad`` (overwritten, not accumulated, as with ``zero_grad(set_to_none=True)``
    before each reference step).  A step with no valid position gives loss 0 and zero gradients,
    as the reference's ``if batch_valid_t > 0`` does."""

    def __init__(self, feats, table, inputs, targets, item_num, num_neg, eps, seed=0, warmup=3):
        L.require_gpu(feats, table, inputs, targets)
        if not (feats.is_leaf and table.is_leaf and feats.requires_grad and table.requires_grad):
            raise RuntimeError("SasTrainStepGraph: feats and table must be leaf tensors requiring grad")
        self.feats, self.table, self.inputs, self.targets = feats, table, inputs, targets
        self.item_num, self.num_neg, self.eps = int(item_num), int(num_neg), float(eps)
        self._check = CHECK or 2 * (inputs.shape[1] + self.num_neg) > self.item_num
        self.seed = torch.tensor([int(seed)], dtype=torch.int64, device=feats.device)
        side = torch.cuda.Stream(device=feats.device)
        side.wait_stream(torch.cuda.current_stream(feats.device))
        with torch.cuda.stream(side):
            for _ in range(warmup):   # allocator / autograd warm-up outside the capture
                feats.grad = table.grad = None
                self._body()
        torch.cuda.current_stream(feats.device).wait_stream(side)
        feats.grad = table.grad = None
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            # detached: the captured autograd graph (and its AccumulateGrad nodes, created on the
            # capture stream) is released, so later eager backwards into the same leaves stay on
            # their own stream
            self.out = tuple(x.detach() for x in self._body())

    def _body(self):
        negs = neg_samples(self.inputs, self.item_num, self.num_neg, seed_tensor=self.seed)
        bl, valid = sampled_bce_loss(self.feats, self.table, self.targets, negs, self.eps)
        (bl / valid.clamp(min=1.0)).backward()   # batch_loss is 0 when nothing is valid
        return bl, valid

    def replay(self):
        self.graph.replay()
        if self._check:   # a row whose negative population may be short: the reference raises
            check_errors(self.feats.device)
        return self.out


class SasTrainGraph:
    """The whole SASRec training step of SASRec/train.py:131-173 -- the transformer forward in
    train mode (dropout on, the drop-in's autograd path), GPU negatives (device-seeded), the fused
    sampled BCE, ``loss = batch_loss / batch_valid_t``, backward and ``optimizer.step()`` --
    captured once as a graph (hipGraph via ``torch.cuda.graph``) and replayed: one launch per step
    instead of ~150 host-issued kernels at the reference's batch of 128.

    ``optimizer`` must be capturable (``torch.optim.Adam(..., capturable=True)``: its step counter
    lives on the device).  ``inputs`` [B, n] and ``targets`` [B, n] are the static batch tensors:
    copy each batch into them before ``replay()``, which returns the static ``(batch_loss,
    batch_valid_t)`` device scalars.  Capture needs a few warm-up steps (allocator, autograd and the
    optimizer's lazily created state); the parameters and the optimizer state are restored
    afterwards, so the first replay is the first real training step.  Dropout draws from torch's
    graph-safe generator (fresh masks each replay)."""

    def __init__(self, model, optimizer, inputs, targets, item_num, num_neg, eps, seed=0, warmup=3,
                 capture=None):
        L.require_gpu(inputs, targets)
        self.model, self.opt = model, optimizer
        if capture is None:   # capture the fused-kernel step; the autograd fallback runs eagerly
            capture = bool(getattr(model, "fused_train", False) and sasrec_train_supported(model, inputs.shape[1]))
        self.inputs, self.targets = inputs, targets
        self.item_num, self.num_neg, self.eps = int(item_num), int(num_neg), float(eps)
        self._check = CHECK or 2 * (inputs.shape[1] + self.num_neg) > self.item_num
        dev = inputs.device
        self.seed = torch.tensor([int(seed)], dtype=torch.int64, device=dev)
        self.graph = None
        if not capture:
            return
        params = [p for g in optimizer.param_groups for p in g["params"]]
        saved_p = [p.detach().clone() for p in params]
        saved_s = {id(p): {k: (v.detach().clone() if torch.is_tensor(v) else v)
                           for k, v in optimizer.state[p].items()} for p in params if p in optimizer.state}
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.out = tuple(x.detach() for x in self._body())
        with torch.no_grad():   # undo the warm-up steps: the first replay is the first step
            for p, s in zip(params, saved_p):
                p.copy_(s)
            for p in params:
                st = optimizer.state.get(p, {})
                old = saved_s.get(id(p))
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if old is not None and torch.is_tensor(old.get(k)):
                            v.copy_(old[k])
                        else:
                            v.zero_()
            self.seed.fill_(int(seed))

    def replay(self):
        """Run one step; returns ``(batch_loss, batch_valid_t)`` (the captured step's static
        tensors).

        The fused-kernel step (``fused_train`` and a shape sasrec_train_supported takes) is one
        captured graph, replayed back to back with no host synchronisation.  With the transformer
        under torch autograd the step runs eagerly instead: back-to-back replays of that graph
        faulted (HSA memory aperture violation) in rocPRIM's unique-by-key partition kernel of the
        item-embedding backward (profiles/r02_train_graph_diag.txt); a graph of captured memsets
        and kernels replays correctly back to back (profiles/r03_graph_memset.txt), so round 2's
        memset-node explanation does not hold, and the fault stays inside that rocPRIM kernel.
        Round 2 synchronised the device after every replay; not capturing that path at all makes
        every path run without a host synchronisation and without the faulting configuration."""
        if self.graph is None:
            out = tuple(x.detach() for x in self._body())
        else:
            self.graph.replay()
            weights_changed()
            out = self.out
        if self._check:   # a row whose negative population may be short: the reference raises
            check_errors(self.inputs.device)
        return out

    def _body(self):
        self.opt.zero_grad(set_to_none=True)
        feats = self.model(self.inputs)                                            # train.py:131
        negs = neg_samples(self.inputs, self.item_num, self.num_neg, seed_tensor=self.seed)   # :142
        bl, valid = sampled_bce_loss(feats, self.model.item_emb.weight, self.targets, negs, self.eps)
        (bl / valid.clamp(min=1.0)).backward()   # :161-172 (batch_loss is 0 when nothing is valid)
        self.opt.step()                                                            # :173
        return bl, valid


class RqTrainGraph:
    """One RQ-VAE training step of RQ-VAE/train.py:108-119 -- ``out, rq_loss, indices =
    model(data)`` (every level's Sinkhorn / argmin assignment on the kernels, dropout on),
    ``compute_loss``, ``loss.backward()``, ``clip_grad_norm_(params, 1.0)`` and ``optimizer.step()``
    -- captured once as a graph (hipGraph via ``torch.cuda.graph``) and replayed: one launch per
    step instead of ~200 host-issued kernels at the reference's batch of 64 (main.py:26).

    ``optimizer`` must be capturable with a tensor learning rate (``torch.optim.AdamW(params,
    lr=torch.tensor(1e-3, device=dev), weight_decay=1e-4, capturable=True)``): its step counter
    and lr live on the device, and a scheduler built on it (``get_linear_schedule_with_warmup``,
    train.py:81-89) writes the new lr in place, so ``scheduler.step()`` after ``replay()`` reaches
    the captured step.  ``inputs`` [B, in_dim] is the static batch: copy each batch into it before
    ``replay()``, which returns the static ``(loss, loss_recon, indices)`` device tensors
    (train.py:120-121's ``.item()`` becomes a device-side sum the caller reads once per epoch).

    A model with ``kmeans_init`` and codebooks not yet initialised is initialised here on
    ``inputs`` -- the reference's first training batch does the same (vq.py:66-67) -- before the
    capture.  Warm-up steps (allocator, autograd, the optimizer's lazily created state) are undone
    afterwards, so the first replay is the first real training step.  Dropout draws from torch's
    graph-safe generator (fresh masks each replay).  On the kernel path (fused MLPs and quantizer)
    replays run back to back (tests/test_rq_train_gpu.py); with the torch modules (``fused_train =
    False``, BatchNorm) the step runs eagerly (SasTrainGraph.replay explains why).  ``capture``
    overrides the choice."""

    def __init__(self, model, optimizer, inputs, max_norm=1.0, use_sk=True, warmup=3, capture=None):
        L.require_gpu(inputs)
        for g in optimizer.param_groups:
            if not g.get("capturable", False) or not torch.is_tensor(g["lr"]):
                raise RuntimeError("RqTrainGraph: the optimizer must be capturable with a tensor lr "
                                   "(e.g. AdamW(params, lr=torch.tensor(1e-3, device=dev), capturable=True))")
        self.model, self.opt, self.inputs = model, optimizer, inputs
        if capture is None:   # capture the kernel path; the torch-module fallback runs eagerly
            capture = bool(getattr(model.encoder, "fused_train", False) and getattr(model.decoder, "fused_train", False)
                           and getattr(model.rq, "fused_train", False) and mlp_train_supported(model.encoder, inputs)
                           and not model.bn)
        self.max_norm, self.use_sk = float(max_norm), bool(use_sk)
        dev = inputs.device
        if model.training and any(not q.initted for q in model.rq.vq_layers):
            with torch.no_grad():   # vq.py:66-67: k-means init on the first batch's residuals
                model(inputs, use_sk=self.use_sk)
        self.graph = None
        if not capture:
            return
        params = [p for g in optimizer.param_groups for p in g["params"]]
        saved_p = [p.detach().clone() for p in params]
        saved_s = {id(p): {k: (v.detach().clone() if torch.is_tensor(v) else v)
                           for k, v in optimizer.state[p].items()} for p in params if p in optimizer.state}
        saved_lr = [g["lr"].detach().clone() for g in optimizer.param_groups]
        # module buffers too: with bn=True every warm-up / capture forward is a train-mode BatchNorm
        # step that moves running_mean / running_var / num_batches_tracked
        bufs = list(model.buffers())
        saved_b = [b.detach().clone() for b in bufs]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        optimizer.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.out = tuple(x.detach() for x in self._body())
        with torch.no_grad():   # undo the warm-up steps: the first replay is the first step
            for p, s in zip(params, saved_p):
                p.copy_(s)
            for p in params:
                st = optimizer.state.get(p, {})
                old = saved_s.get(id(p))
                for k, v in st.items():
                    if torch.is_tensor(v):
                        if old is not None and torch.is_tensor(old.get(k)):
                            v.copy_(old[k])
                        else:
                            v.zero_()
            for g, lr in zip(optimizer.param_groups, saved_lr):
                g["lr"].copy_(lr)
            for b, sb in zip(bufs, saved_b):
                b.copy_(sb)

    def replay(self):
        """Run one step; returns ``(loss, loss_recon, indices)`` (the captured step's static tensors).
        The kernel path is one captured graph replayed back to back; the torch-module fallback runs
        eagerly (SasTrainGraph.replay explains why)."""
        if self.graph is None:
            return tuple(x.detach() for x in self._body())
        self.graph.replay()
        weights_changed()   # the captured AdamW step moved the weights without a version bump
        return self.out

    def _body(self):
        self.opt.zero_grad(set_to_none=True)
        out, rq_loss, indices = self.model(self.inputs, use_sk=self.use_sk)           # train.py:113
        loss, loss_recon = self.model.compute_loss(out, rq_loss, xs=self.inputs)     # :114
        loss.backward()                                                              # :116
        torch.nn.utils.clip_grad_norm_(self.model.parameters(), self.max_norm)       # :117
        self.opt.step()                                                              # :118
        return loss, loss_recon, indices


class _RqQuantTrain(torch.autograd.Function):
    """ResidualVectorQuantizer.forward under autograd (rq.py:39-56, vq.py:63-99) in one launch
    forward and two backward: the assignment of every level (Sinkhorn or argmin), x_q and the mse
    numerators (gr_rq_quantize_sk_train_f32); dz and every codebook's gradient
    (gr_rq_quantize_sk_train_bwd_f32)."""

    @staticmethod
    def forward(ctx, z, beta, sk_eps, sk_iters, *codebooks):
        n, e = z.shape
        dev = z.device
        Ks = [c.shape[0] for c in codebooks]
        lib = L.lib()
        ks_c = L.i32_array(Ks)
        eps_c = (ctypes.c_double * len(codebooks))(*[float(v) for v in sk_eps])
        nbytes = lib.gr_rq_encode_sk_workspace_bytes(n, e, len(codebooks), ks_c)
        wsp = L.workspace(nbytes, dev)
        idx = torch.empty((n, len(codebooks)), dtype=torch.int64, device=dev)
        xq = torch.empty((n, e), dtype=torch.float32, device=dev)
        sq = torch.empty((n, len(codebooks)), dtype=torch.float32, device=dev)
        with L.on(dev):
            L.check(lib.gr_rq_quantize_sk_train_f32(L.ptr(z), n, e, len(codebooks), ks_c, L.ptr_array(codebooks),
                                                    eps_c, int(sk_iters), L.ptr(_group_ptr([n], dev)), 1,
                                                    L.ptr(idx), L.ptr(xq), L.ptr(sq), L.ptr(wsp), nbytes,
                                                    L.stream_of(dev)), "gr_rq_quantize_sk_train_f32")
        m = sq.sum(0) / float(n * e)                       # vq.py:88-89: mse per level
        rq_loss = (m + beta * m).mean()                    # vq.py:90, rq.py:51
        ctx.save_for_backward(z, idx, *codebooks)
        ctx.beta = float(beta)
        ctx.mark_non_differentiable(idx)
        return xq, rq_loss, idx

    @staticmethod
    def backward(ctx, g_xq, g_rq, _g_idx):
        z, idx, *codebooks = ctx.saved_tensors
        n, e = z.shape
        dev = z.device
        g_rq = (g_rq if g_rq is not None else torch.zeros((), device=dev)).to(torch.float32).contiguous()
        g_xq = g_xq.contiguous() if g_xq is not None else None
        dz = torch.empty_like(z)
        dcs = [torch.empty_like(c) for c in codebooks]
        with L.on(dev):
            L.check(L.lib().gr_rq_quantize_sk_train_bwd_f32(
                L.ptr(z), n, e, len(codebooks), L.i32_array([c.shape[0] for c in codebooks]),
                L.ptr_array(codebooks), L.ptr(idx), L.ptr(g_xq) if g_xq is not None else None, L.ptr(g_rq),
                ctypes.c_float(ctx.beta), L.ptr(dz), L.ptr_array(dcs), L.stream_of(dev)),
                "gr_rq_quantize_sk_train_bwd_f32")
        return (dz, None, None, None, *dcs)


def rq_quantize_train(z, codebooks, beta, sk_eps, sk_iters):
    """``(x_q, rq_loss, indices)`` of ResidualVectorQuantizer.forward(z, use_sk) in training
    (rq.py:39-56): differentiable in ``z`` and every codebook, the whole batch one Sinkhorn group
    per level where ``sk_eps[l] > 0`` (vq.py:76-84), the plain argmin elsewhere."""
    L.require_gpu(z, *codebooks)
    if z.dtype != torch.float32 or any(c.dtype != torch.float32 for c in codebooks):
        raise TypeError("rq_quantize_train takes float32 tensors")
    if any(c.shape[0] > 1024 for c in codebooks):
        raise RuntimeError("rq_quantize_train: codebooks of at most 1024 codes")
    return _RqQuantTrain.apply(z.contiguous(), float(beta), [float(v) for v in sk_eps], int(sk_iters),
                               *[c.contiguous() if not c.is_contiguous() else c for c in codebooks])


class _MlpTrain(torch.autograd.Function):
    """MLPLayers.forward in train mode (RQ-VAE/models/layers.py:18-43) and its backward on the
    kernels of rq_mlp_train.hip: the input dropout, then one launch per layer forward (bias, ReLU,
    and the next layer's dropout in the epilogue) and one per layer backward (weight and bias
    gradients and the input gradient with the ReLU and dropout masks folded in)."""

    @staticmethod
    def forward(ctx, x, p, snap, *params):
        ws, bs = params[0::2], params[1::2]
        n = len(ws)
        M = x.shape[0]
        dev = x.device
        dims = [x.shape[1]] + [w.shape[0] for w in ws]
        outs = [torch.empty((M, dd), dtype=torch.float32, device=dev) for dd in dims[1:]]
        xd0 = torch.empty_like(x) if p > 0 else x
        with L.on(dev):
            L.check(L.lib().gr_mlp_train_fwd_f32(L.ptr(x), M, n, L.i32_array(dims), L.ptr_array(ws),
                                                 L.ptr_array(bs), float(p), L.ptr(snap),
                                                 L.ptr(xd0) if p > 0 else None, L.ptr_array(outs),
                                                 L.stream_of(dev)), "gr_mlp_train_fwd_f32")
        ctx.save_for_backward(xd0, snap, *outs[:-1], *ws)
        ctx.p, ctx.n = float(p), n
        return outs[-1]

    @staticmethod
    def backward(ctx, dout):
        xd0, snap, *rest = ctx.saved_tensors
        n = ctx.n
        acts, ws = [xd0] + rest[:n - 1], rest[n - 1:]
        M = xd0.shape[0]
        dev = xd0.device
        dz = dout.contiguous().float()
        gw, gb = [None] * n, [None] * n
        with L.on(dev):
            for i in reversed(range(n)):
                K, N = acts[i].shape[1], ws[i].shape[0]
                dW = torch.empty_like(ws[i])
                db = torch.empty((N,), dtype=torch.float32, device=dev)
                dX = (torch.empty((M, K), dtype=torch.float32, device=dev)
                      if i > 0 or ctx.needs_input_grad[0] else None)
                L.check(L.lib().gr_mlp_train_bwd_layer_f32(
                    L.ptr(acts[i]), M, K, L.ptr(ws[i]), N, L.ptr(dz), 1 if i > 0 else 2, ctx.p, L.ptr(snap), 0,
                    L.ptr(dW), L.ptr(db), L.ptr(dX), L.stream_of(dev)), "gr_mlp_train_bwd_layer_f32")
                gw[i], gb[i] = dW, db
                dz = dX
        grads = [dz if ctx.needs_input_grad[0] else None, None, None]
        for w, b in zip(gw, gb):
            grads += [w, b]
        return tuple(grads)


def mlp_train_supported(mlp, x):
    lin = mlp.linears()
    return (x.is_cuda and x.dim() == 2 and x.dtype == torch.float32 and not mlp.use_bn
            and (mlp.act == "relu" or len(lin) == 1) and all(m.bias is not None for m in lin)
            and x.shape[1] == lin[0].weight.shape[1])


def mlp_train(x, mlp):
    """``mlp.mlp_layers(x)`` under autograd (RQ-VAE/models/layers.py:42-43 as RQVAE.forward calls it
    in training, RQ-VAE/train.py:113): dropout (train mode), Linear, ReLU on the fused training
    kernels, differentiable in ``x`` and every Linear's weight and bias.  Dropout masks come from the
    device's seed word (``dropout_seed``), so a captured step replays with fresh masks."""
    L.require_gpu(x)
    p = float(mlp.dropout) if mlp.training else 0.0
    seed = dropout_seed(x.device)
    snap = seed + 0              # this call's masks (its backward reads the same word)
    seed.add_(1)
    params = []
    for m in mlp.linears():
        params += [m.weight, m.bias]
    return _MlpTrain.apply(x.contiguous(), p, snap, *params)
