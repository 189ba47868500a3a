"""Dependent-chain latency of v_mfma_f32_16x16x4_f32 / v_mfma_f32_32x32x2_f32 (cycles per MFMA when
each one accumulates into the previous one's result) and the shader clock (s_memtime over
s_memrealtime at 100 MHz) of a small launch: cold, and right after 0.5 s of back-to-back launches.
Builds scripts/micro/libmfma_chain.so from mfma_chain.hip if it is missing."""
import ctypes
import os
import subprocess
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
so = os.path.join(HERE, "libmfma_chain.so")
if not os.path.exists(so):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-shared", "-fPIC", "--offload-arch=gfx950",
                    os.path.join(HERE, "mfma_chain.hip"), "-o", so], check=True)
lib = ctypes.CDLL(so)
lib.run_chain.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
out = torch.zeros(64 * 256, device="cuda")
clk = torch.zeros(2 * 256, dtype=torch.int64, device="cuda")
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def run(kind, blocks, iters):
    lib.run_chain(kind, out.data_ptr(), clk.data_ptr(), blocks, iters, st)
    torch.cuda.synchronize()
    c = clk[: 2 * blocks].view(-1, 2).double()
    cyc = c[:, 0].mean().item()
    ghz = (c[:, 0] / c[:, 1] * 0.1).mean().item()
    return cyc / iters, ghz, c[:, 1].mean().item() * 10 / iters   # cycles / MFMA, GHz, ns / MFMA


for label in ("cold", "warm"):
    if label == "warm":
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.5:
            lib.run_chain(0, out.data_ptr(), clk.data_ptr(), 256, 20000, st)
        torch.cuda.synchronize()
    for kind, name in ((0, "16x16x4"), (1, "32x32x2")):
        for blocks, iters in ((1, 64), (4, 64), (4, 4096), (256, 4096)):
            cpm, ghz, ns = run(kind, blocks, iters)
            print(f"{label}: {name} chain of {iters:5d} on {blocks:3d} waves: {cpm:6.1f} cycles / {ns:6.1f} ns per "
                  f"dependent MFMA, shader clock {ghz:5.3f} GHz", flush=True)
