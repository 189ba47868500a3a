"""A/B of the scoring kernel's diagnostic ablation builds (build.py build_stamps variants):
time gr_score_f32 at config C3 (B=2048, 100001 rows, d=64) with HIP events.

    python scripts/ab_score.py [suffix ...]      (suffix '' = the product library)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib  # noqa: E402

B, ROWS = int(os.environ.get("AB_B", 2048)), int(os.environ.get("AB_ROWS", 100001))
D = int(os.environ.get("AB_D", 64))
LD = int(os.environ.get("AB_LD", ROWS))   # row stride of the logits (ROWS = the reference layout)
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
h = torch.randn((B, D), generator=g, device=dev)
t = torch.randn((ROWS, D), generator=g, device=dev)
out = torch.empty((B, LD), device=dev)
base = os.path.dirname(_lib.LIB_PATH)
for suf in (sys.argv[1:] or [""]):
    path = os.path.join(base, "libgr_amd.so" if suf == "" else f"libgr_amd_stamps{suf}.so")
    lib = ctypes.CDLL(path)
    fn = lib.gr_score_f32
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                   ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    call = lambda: fn(h.data_ptr(), B, D, t.data_ptr(), ROWS, out.data_ptr(), LD, st)
    for _ in range(3):
        assert call() == 0
    lib.gr_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
    if os.environ.get("AB_FLAGS") is not None:
        assert lib.gr_set_option(b"score_flags", int(os.environ["AB_FLAGS"])) == 0
        suf = (suf or "") + f"flags{os.environ['AB_FLAGS']}"
    if os.environ.get("AB_IMPL") is not None:
        assert lib.gr_set_option(b"score_impl", int(os.environ["AB_IMPL"])) == 0
        suf = (suf or "") + f"impl{os.environ['AB_IMPL']}"
    if os.environ.get("AB_UBM") is not None:
        assert lib.gr_set_option(b"score_ubmajor", int(os.environ["AB_UBM"])) == 0
        suf = (suf or "") + f"ubm{os.environ['AB_UBM']}"
    abl = int(os.environ.get("AB_ABLATE", 0))
    if abl:
        lib.gr_set_option.argtypes = [ctypes.c_char_p, ctypes.c_int64]
        assert lib.gr_set_option(b"score_ablate", abl) == 0
        suf = (suf or "") + f"ablate{abl}"
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = int(os.environ.get("AB_REPS", 20))
    e0.record()
    for _ in range(reps):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(f"ld={LD} {suf or 'product':12s} {ms * 1e3:8.1f} us  {2 * B * ROWS * D / ms / 1e9:7.1f} TF/s  "
          f"{B * ROWS * 4 / ms / 1e6:7.0f} GB/s logits", flush=True)
# write-bandwidth reference: torch fill of the same logits buffer
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
out.fill_(1.0)
e0.record()
for _ in range(20):
    out.fill_(1.0)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 20
print(f"{'torch fill':12s} {ms * 1e3:8.1f} us  {B * ROWS * 4 / ms / 1e6:7.0f} GB/s", flush=True)
