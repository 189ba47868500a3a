"""Run scripts/micro/store_pattern.hip (build: hipcc -shared -fPIC --offload-arch=gfx950)."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libstore_pattern.so"))
lib.run_store_pattern.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
B, ld = 2048, 100032
out = torch.empty((B, ld), device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for L in (1, 2, 4, 8):
    for _ in range(3):
        lib.run_store_pattern(out.data_ptr(), ld, ld, L, st)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        lib.run_store_pattern(out.data_ptr(), ld, ld, L, st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"L={L} ({128 * L} B per row visit): {ms * 1e3:7.1f} us  {B * ld * 4 / ms / 1e6:7.0f} GB/s", flush=True)
