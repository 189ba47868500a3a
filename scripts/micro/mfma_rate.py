"""Run scripts/micro/mfma_rate.hip (built into scripts/micro/libmfma_rate.so by
``hipcc -O3 -shared -fPIC --offload-arch=gfx950``): sustained fp32 MFMA TFLOP/s on the whole chip
and the effective shader clock, per (waves per workgroup, chains per wave)."""
import ctypes
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_rate.so"))
lib.run_mfma_rate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_void_p]
lib.run_mfma_rate_lds.argtypes = lib.run_mfma_rate.argtypes
cus = torch.cuda.get_device_properties(0).multi_processor_count
out = torch.zeros(1024, device="cuda")
clk = torch.zeros(2 * cus, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
iters = 20000
for fn, tag in ((lib.run_mfma_rate, "registers"), (lib.run_mfma_rate_lds, "A from LDS")):
  for waves, chains in [(4, 1), (4, 2), (4, 4), (8, 1), (8, 2), (8, 4), (16, 1)]:
    for _ in range(3):
        fn(out.data_ptr(), clk.data_ptr(), cus, waves, chains, iters, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn(out.data_ptr(), clk.data_ptr(), cus, waves, chains, iters, st)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    flop = cus * waves * chains * iters * 32 * 32 * 2 * 2
    c = clk.view(-1, 2).double()
    ghz = (c[:, 0] / c[:, 1] * 0.1).mean().item()   # s_memrealtime ticks at 100 MHz
    cyc = (c[:, 0].mean().item()) / (iters * chains * waves / 4)
    print(f"{tag:10s} waves/WG {waves:2d} chains/wave {chains}: {flop / ms / 1e9:7.1f} TFLOP/s  "
          f"({flop / ms / 1e9 / 157.3:5.3f} of 157.3)  shader clock {ghz:5.3f} GHz  "
          f"{cyc:6.1f} cycles per MFMA per SIMD", flush=True)
