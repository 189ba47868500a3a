"""Run scripts/micro/mfma_valu.hip (built into scripts/micro/libmfma_valu.so by
``hipcc -O3 -shared -fPIC --offload-arch=gfx950``): whole-chip fp32 flop rate of v_mfma_f32_32x32x2_f32
chains with V v_fma_f32 per MFMA beside them -- in the same wave (mode 0) or in partner waves on the
same SIMD (mode 1) -- to learn whether VALU fma work adds to the MFMA pipe's 157.3 TFLOP/s."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_valu.so"))
lib.run_mfma_valu.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
cus = torch.cuda.get_device_properties(0).multi_processor_count
out = torch.zeros(1024, device="cuda")
clk = torch.zeros(2 * cus, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
iters = 20000
CH = 2
for mode in (0, 1):
    for waves in (4, 8):
        if mode == 1 and waves == 4:
            continue
        for V in (0, 2, 4, 6, 8, 12, 16):
            for _ in range(2):
                lib.run_mfma_valu(out.data_ptr(), clk.data_ptr(), cus, waves, V, mode, iters, st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            lib.run_mfma_valu(out.data_ptr(), clk.data_ptr(), cus, waves, V, mode, iters, st)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            mw = waves if mode == 0 else waves // 2   # waves issuing MFMAs
            vw = waves if mode == 0 else waves // 2   # waves issuing VALU fmas
            mflop = cus * mw * CH * iters * 32 * 32 * 2 * 2
            vflop = cus * vw * CH * iters * V * 64 * 2
            c = clk.view(-1, 2).double()
            ghz = (c[:, 0] / c[:, 1] * 0.1).mean().item()
            print(f"mode {mode} waves/WG {waves} V/MFMA {V:2d}: MFMA {mflop / ms / 1e9:6.1f} + VALU "
                  f"{vflop / ms / 1e9:6.1f} = {(mflop + vflop) / ms / 1e9:6.1f} TFLOP/s "
                  f"({(mflop + vflop) / ms / 1e9 / 157.3:5.3f} of 157.3)  clock {ghz:5.3f} GHz", flush=True)
