"""ctypes binding of oracle/rq_exact.c, the exact-order restatement of ``RQVAE.get_indices`` —
TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Every fp32 rounding of the reference's CPU run (MKL sgemm k-blocking, ATen's vectorised row sums,
vq.py:71-75's association order) is spelled out in rq_exact.c, so the result does not depend on the
host's BLAS.  Pinned against every RQ golden fixture by tests/test_rq_exact_oracle.py.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "lib", "librq_exact.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
        _lib.rqx_kblock.restype = ctypes.c_int
        for f in ("rqx_encode_m", "rqx_quantize_m", "rqx_linear", "rqx_mlp_m", "rqx_plan", "rqx_plan_pinned"):
            getattr(_lib, f).restype = ctypes.c_int
    return _lib


def _f(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _p(a):
    return a.ctypes.data_as(_f32p)


def _ptrs(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def _threads(threads):
    if threads:
        return int(threads)
    return min(16, len(os.sched_getaffinity(0)))


def kblock(k):
    return lib().rqx_kblock(int(k))


PLAN_KINDS = {0: "chain", 1: "gemv16", 2: "small16"}


def plan(m, k, n):
    """MKL's accumulation order for a call of ``m`` rows, inner size ``k``, ``n`` outputs:
    (kind, block width, pinned) -- see rq_exact.c rqx_plan / rqx_plan_pinned."""
    kb = ctypes.c_int(0)
    kind = lib().rqx_plan(ctypes.c_int64(int(m)), int(k), int(n), ctypes.byref(kb))
    return PLAN_KINDS[kind], kb.value, bool(lib().rqx_plan_pinned(ctypes.c_int64(int(m)), int(k), int(n)))


def linear(x, w, b=None, act="none"):
    """One reference ``F.linear`` call on the rows of ``x`` (the order depends on their count)."""
    x, w = _f(x), _f(w)
    b = None if b is None else _f(b)
    y = np.empty((x.shape[0], w.shape[0]), np.float32)
    rc = lib().rqx_linear(_p(x), ctypes.c_int64(x.shape[0]), x.shape[1], _p(w), w.shape[0],
                          None if b is None else _p(b), {"none": 0, "relu": 1, "leakyrelu": 2}[act], _p(y))
    if rc:
        raise ValueError("rq_exact.linear: bad arguments")
    return y


def rowsq(x):
    x = _f(x)
    out = np.empty(x.shape[0], np.float32)
    lib().rqx_rowsq_rows(_p(x), ctypes.c_int64(x.shape[0]), x.shape[1], _p(out))
    return out


def encode(x, weights, biases, codebooks, with_detail=False, threads=None, call_m=None):
    """get_indices(x) with encoder ``weights``/``biases`` ([out, in] / [out]) and ``codebooks``
    ([K, e] per level) -> idx [n, L] int64 (and z, best distance, best/second gap with detail).
    All rows are ONE reference call of ``call_m`` rows (default: n) -- MKL's order depends on it."""
    x = _f(x)
    ws = [_f(w) for w in weights]
    bs = [_f(b) for b in biases]
    cbs = [_f(c) for c in codebooks]
    n, L = x.shape[0], len(cbs)
    dims = (ctypes.c_int * (len(ws) + 1))(*([x.shape[1]] + [w.shape[0] for w in ws]))
    K = (ctypes.c_int * L)(*[c.shape[0] for c in cbs])
    idx = np.empty((n, L), np.int64)
    e = ws[-1].shape[0]
    z = np.empty((n, e), np.float32) if with_detail else None
    best = np.empty((n, L), np.float32) if with_detail else None
    gap = np.empty((n, L), np.float32) if with_detail else None
    rc = lib().rqx_encode_m(_p(x), ctypes.c_int64(n), len(ws), dims, _ptrs(ws), _ptrs(bs), L, K, _ptrs(cbs),
                            idx.ctypes.data_as(_i64p), None if z is None else _p(z),
                            None if best is None else _p(best), None if gap is None else _p(gap),
                            _threads(threads), ctypes.c_int64(call_m or n))
    if rc:
        raise ValueError("rq_exact.encode: bad arguments")
    return (idx, z, best, gap) if with_detail else idx


def quantize(z, codebooks, with_detail=False, threads=None, call_m=None):
    z = _f(z)
    cbs = [_f(c) for c in codebooks]
    n, L = z.shape[0], len(cbs)
    K = (ctypes.c_int * L)(*[c.shape[0] for c in cbs])
    idx = np.empty((n, L), np.int64)
    best = np.empty((n, L), np.float32) if with_detail else None
    gap = np.empty((n, L), np.float32) if with_detail else None
    lib().rqx_quantize_m(_p(z), ctypes.c_int64(n), z.shape[1], L, K, _ptrs(cbs), idx.ctypes.data_as(_i64p),
                         None if best is None else _p(best), None if gap is None else _p(gap), _threads(threads),
                         ctypes.c_int64(call_m or n))
    return (idx, best, gap) if with_detail else idx


def mlp(x, weights, biases, bn=None, act="relu", threads=None, call_m=None):
    """MLPLayers.forward (eval) in the reference's CPU order: ``bn`` = None or (means, vars, weights,
    biases, eps) of the BatchNorm1d after every Linear but the last; act relu / leakyrelu / none."""
    x = _f(x)
    ws = [_f(w) for w in weights]
    bs = [_f(b) for b in biases]
    n = x.shape[0]
    dims = (ctypes.c_int * (len(ws) + 1))(*([x.shape[1]] + [w.shape[0] for w in ws]))
    z = np.empty((n, ws[-1].shape[0]), np.float32)
    arrs = [None] * 4
    eps = 0.0
    keep = []
    if bn is not None:
        means, vars_, bws, bbs, eps = bn
        for j, grp in enumerate((means, vars_, bws, bbs)):
            if grp is None or all(t is None for t in grp):
                continue
            ts = [_f(t) for t in grp]
            keep.append(ts)
            arrs[j] = _ptrs(ts)
    rc = lib().rqx_mlp_m(_p(x), ctypes.c_int64(n), len(ws), dims, _ptrs(ws), _ptrs(bs), *arrs,
                         ctypes.c_float(eps), {"none": 0, "relu": 1, "leakyrelu": 2}[act], _p(z), _threads(threads),
                         ctypes.c_int64(call_m or n))
    if rc:
        raise ValueError("rq_exact.mlp: bad arguments")
    return z


def encode_batches(x, weights, biases, codebooks, bs=64, threads=None):
    """The reference's DataLoader loop (RQ-VAE/infer.py:84-95, generate_code.py:78-88): one
    get_indices call per ``bs`` rows, the tail call with its own (short) row count."""
    x = _f(x)
    parts = [encode(x[i:i + bs], weights, biases, codebooks, threads=threads) for i in range(0, x.shape[0], bs)]
    return np.concatenate(parts) if parts else np.zeros((0, len(codebooks)), np.int64)
