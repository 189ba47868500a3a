"""Run scripts/micro/attn_shape.hip (built into scripts/micro/libattn_shape.so by
``hipcc -O3 -shared -fPIC --offload-arch=gfx950``): cycles per MFMA per SIMD of the per-wave
attention kernel's MFMA shape at one wave per SIMD (4 x CUs one-wave workgroups)."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libattn_shape.so"))
lib.run_attn_shape.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p]
cus = torch.cuda.get_device_properties(0).multi_processor_count
blocks = 4 * cus
out = torch.zeros(64, device="cuda")
clk = torch.zeros(2 * blocks, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
iters = 2000
names = {0: "S chain (64 dep.) + PV (4 x 16, B from S)", 1: "S chain only (64 dep.)", 2: "PV only (B from regs)"}
mfmas = {0: 128, 1: 64, 2: 64}
for mode in (0, 1, 2):
    for _ in range(3):
        lib.run_attn_shape(out.data_ptr(), clk.data_ptr(), blocks, mode, iters, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lib.run_attn_shape(out.data_ptr(), clk.data_ptr(), blocks, mode, iters, st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    c = clk.view(-1, 2).double()
    ghz = (c[:, 0] / c[:, 1] * 0.1).mean().item()
    cyc = c[:, 0].mean().item() / (iters * mfmas[mode])
    flop = blocks * iters * mfmas[mode] * 32 * 32 * 2 * 2
    print(f"{names[mode]:45s}: {cyc:6.1f} cycles per MFMA per SIMD, clock {ghz:5.3f} GHz, "
          f"{flop / ms / 1e9:7.1f} TFLOP/s", flush=True)
