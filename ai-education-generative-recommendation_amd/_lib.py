"""ctypes binding of libgr_amd.so (the C ABI declared in include/gr_amd.h).

The library is built in-tree by ``build.py`` (``__graft_entry__.build()``).  There is no CPU or
PyTorch fallback: if the library is missing, or a tensor is not on a ROCm device, the call raises.
"""
import ctypes
import os

import torch

_PKG = os.path.dirname(os.path.abspath(__file__))
# GR_AMD_LIB: another in-tree build of the same ABI (A/B variants from scripts/build_variant.sh)
LIB_PATH = os.environ.get("GR_AMD_LIB") or os.path.join(_PKG, "lib", "libgr_amd.so")

GR_ACT_NONE = 0
GR_ACT_RELU = 1
GR_ACT_SIGMOID = 2
GR_ACT_TANH = 3
GR_ACT_LEAKYRELU = 4
GR_MAX_LEVELS = 8
GR_MAX_LINEAR = 8

_c_int_p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_sz = ctypes.c_size_t
_f32 = ctypes.c_float


class SasrecParams(ctypes.Structure):
    """Mirror of ``gr_sasrec_params`` (include/gr_amd.h)."""
    _fields_ = [("d", _i32), ("n_blocks", _i32), ("n_heads", _i32), ("mlp", _i32),
                ("max_len", _i32), ("eps", _f32), ("item_rows", _i64),
                ("item_emb", _vp), ("pos_emb", _vp),
                ("attn_ln_w", _vp), ("attn_ln_b", _vp), ("in_proj_w", _vp), ("in_proj_b", _vp),
                ("out_proj_w", _vp), ("out_proj_b", _vp), ("ffn_ln_w", _vp), ("ffn_ln_b", _vp),
                ("ffn1_w", _vp), ("ffn1_b", _vp), ("ffn2_w", _vp), ("ffn2_b", _vp),
                ("last_ln_w", _vp), ("last_ln_b", _vp)]


class SasrecTrainBufs(ctypes.Structure):
    """Mirror of ``gr_sasrec_train_bufs`` (include/gr_amd.h)."""
    _fields_ = [(f, _vp) for f in ("xin", "hs", "qkv", "prob", "os", "x1", "fs", "zs", "us", "xl", "g_vec")]


# (name, restype, argtypes) for every entry point of include/gr_amd.h
SIGNATURES = {
    "gr_version": (ctypes.c_char_p, []),
    "gr_last_error": (ctypes.c_char_p, []),
    "gr_set_option": (ctypes.c_int, [ctypes.c_char_p, _i64]),
    "gr_get_option": (_i64, [ctypes.c_char_p]),
    "gr_linear_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _vp, _i64, _i32, _vp, _i64, _vp]),
    "gr_rq_codebook_norms_f32": (ctypes.c_int, [_vp, _i32, _i32, _vp, _vp]),
    "gr_rq_quantize_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "gr_rq_encode_workspace_bytes": (_sz, [_i64, _i32, _vp, _i32, _vp]),
    "gr_rq_encode_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp,
                                        _vp, _vp, _vp, _sz, _vp]),
    "gr_rq_encoder_pack_floats": (_sz, [_i32, _vp]),
    "gr_rq_encoder_pack_f32": (ctypes.c_int, [_i32, _vp, _vp, _vp, _vp]),
    "gr_rq_encode_packed_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp,
                                               _vp, _vp, _vp, _vp, _sz, _vp]),
    "gr_rq_mlp_workspace_bytes": (_sz, [_i64, _i32, _vp]),
    "gr_rq_mlp_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "gr_mlp_exact_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32, _i32,
                                        _vp, _vp, _sz, _vp]),
    "gr_mlp_exact_groups_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f32,
                                               _i32, _vp, _i64, _vp, _vp]),
    "gr_mkl_plan": (_i32, [_i64, _i32, _i32, _c_int_p, _c_int_p]),
    "gr_rq_encode_sk_workspace_bytes": (_sz, [_i64, _i32, _i32, _vp]),
    "gr_rq_encode_sk_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _i64,
                                           _vp, _vp, _sz, _vp]),
    "gr_mlp_train_fwd_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _vp, _vp, _f32, _vp, _vp, _vp, _vp]),
    "gr_mlp_train_bwd_layer_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i32, _vp, _i32, _f32, _vp, _i32,
                                                  _vp, _vp, _vp, _vp]),
    "gr_rq_quantize_sk_train_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _i32, _vp, _i64,
                                                   _vp, _vp, _vp, _vp, _sz, _vp]),
    "gr_rq_quantize_sk_train_bwd_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp, _vp, _vp, _vp, _f32,
                                                       _vp, _vp, _vp]),
    "gr_sasrec_workspace_bytes": (_sz, [ctypes.POINTER(SasrecParams), _i64, _i32]),
    "gr_sasrec_forward_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _vp,
                                             _i32, _vp, _sz, _vp, _vp]),
    "gr_sasrec_predict_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _vp,
                                             _vp, _sz, _vp, _vp]),
    "gr_sasrec_predict_ld_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _vp,
                                                _i64, _vp, _sz, _vp, _vp]),
    "gr_sasrec_rank_workspace_bytes": (_sz, [ctypes.POINTER(SasrecParams), _i64, _i32]),
    "gr_sasrec_rank_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _vp, _i32, _vp, _vp,
                                          _sz, _vp, _sz, _vp, _vp]),
    "gr_sasrec_train_vec_width": (_i32, [ctypes.POINTER(SasrecParams), _i32]),
    "gr_sasrec_train_fwd_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _f32,
                                               ctypes.c_uint64, _vp, ctypes.POINTER(SasrecTrainBufs), _vp,
                                               _vp, _vp]),
    "gr_sasrec_train_bwd_f32": (ctypes.c_int, [ctypes.POINTER(SasrecParams), _vp, _i64, _i32, _f32,
                                               ctypes.c_uint64, _vp, ctypes.POINTER(SasrecTrainBufs), _vp,
                                               _vp, _vp]),
    "gr_score_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _i64, _vp]),
    "gr_sampled_bce_fwd_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp, _vp, _i32, _f32,
                                              _vp, _vp, _vp, _vp, _vp]),
    "gr_neg_samples": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i32, ctypes.c_uint64, _vp, _vp, _vp]),
    "gr_neg_samples_dseed": (ctypes.c_int, [_vp, _i64, _i32, _i64, _i32, ctypes.c_uint64, _vp, _vp, _vp, _vp]),
    "gr_sampled_bce_bwd_f32": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _i64, _vp, _vp, _i32, _vp,
                                              _vp, _vp, _vp, _vp]),
    "gr_rank_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _i32, _vp, _vp]),
    "gr_count_gt_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _vp, _vp, _vp]),
    "gr_topk_workspace_bytes": (_sz, [_i64, _i64, _i32]),
    "gr_topk_f32": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "gr_score_pairs_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _vp, _vp]),
    "gr_score_count_gt_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _vp]),
    "gr_score_count_workspace_bytes": (_sz, [_i64]),
    "gr_score_count_gt_ws_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _vp, _i32, _vp, _vp, _sz, _vp]),
    "gr_merge_topk_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp]),
    "gr_merge_topk_packed": (ctypes.c_int, [_vp, _i32, _i64, _i32, _i32, _vp, _vp, _vp]),
    "gr_score_topk_workspace_bytes": (_sz, [_i64, _i32, _i64, _i32]),
    "gr_score_topk_f32": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _i64, _i32, _i32, _vp, _vp, _vp,
                                         _vp, _vp, _sz, _vp]),
}

_lib = None


def lib():
    """Load (once) and return the ctypes handle; raises if the library has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"gr_amd: {LIB_PATH} is missing - run __graft_entry__.build() "
                               "(there is no CPU fallback)")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().gr_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (code {rc}): {msg}")


def require_gpu(*tensors):
    """The product path runs only on a ROCm device: refuse CPU tensors loudly."""
    for t in tensors:
        if not t.is_cuda:
            raise RuntimeError("gr_amd kernels run on a ROCm GPU only (tensor on "
                               f"{t.device}); there is no CPU fallback")


def ptr(t):
    """Device address of ``t`` as a plain int (the argtypes convert it; None: NULL)."""
    return t.data_ptr() if t is not None else None


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(device):
    """Handle of ``device``'s current stream (int) -- the stream every call enqueues on."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if _raw_stream is not None:
        return _raw_stream(idx)
    return torch.cuda.current_stream(idx).cuda_stream


class _NoGuard:
    __slots__ = ()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_NO_GUARD = _NoGuard()


def on(device):
    """Device guard for a launch on ``device``: a no-op when it is already the current device (the
    common case; torch.cuda.device's set / restore costs microseconds per call at the reference's
    batch sizes), torch.cuda.device otherwise."""
    if device.index is None or device.index == torch.cuda.current_device():
        return _NO_GUARD
    return torch.cuda.device(device)


def ptr_array(tensors):
    """Host array of device pointers (``const float* const*``)."""
    arr = (ctypes.c_void_p * len(tensors))(*[t.data_ptr() for t in tensors])
    return arr


def i32_array(values):
    return (ctypes.c_int32 * len(values))(*values)


def workspace(nbytes, device):
    """Caller-owned scratch from the PyTorch caching allocator (the library never allocates)."""
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def as_f32(t):
    """Contiguous fp32 view (the kernels are fp32 end to end, like the reference)."""
    if t.dtype != torch.float32:
        raise TypeError(f"gr_amd kernels take float32 tensors, got {t.dtype}")
    return t.contiguous()


def set_option(name, value):
    """gr_set_option (include/gr_amd.h): process-wide path / tuning switches."""
    check(lib().gr_set_option(name.encode(), int(value)), "gr_set_option")


def get_option(name):
    return int(lib().gr_get_option(name.encode()))
