"""Rounding sequence of the f32-input MFMAs (scripts/micro/mfma_order.hip, built into
scripts/micro/libmfma_order.so by ``hipcc -O3 -shared -fPIC --offload-arch=gfx950``): compare each
chain's result with fmaf chains in candidate k orders (emulated in float64 then rounded; exact for
one fma).  Prints the fraction of outputs each candidate reproduces bit for bit."""
import ctypes
import os

import numpy as np
import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmfma_order.so"))
lib.run_chain.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                          ctypes.c_void_p]


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(np.float32)


rng = np.random.default_rng(0)
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for shape, kk in ((16, 4), (32, 2)):
    M = shape
    for trial in range(3):
        S = 48
        A = rng.standard_normal((S, M, kk), dtype=np.float32) * rng.uniform(0.01, 10, (S, M, kk)).astype(np.float32)
        B = rng.standard_normal((S, kk, M), dtype=np.float32)
        D = torch.empty((M, M), device="cuda")
        At, Bt = torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda()
        lib.run_chain(shape, At.data_ptr(), Bt.data_ptr(), S, D.data_ptr(), st)
        torch.cuda.synchronize()
        got = D.cpu().numpy()
        res = {}
        for name, order in (("k ascending", list(range(kk))), ("k descending", list(range(kk))[::-1])):
            acc = np.zeros((M, M), np.float32)
            for s in range(S):
                for k in order:
                    acc = fma(A[s][:, k][:, None], B[s][k][None, :], acc)
            res[name] = float(np.mean(acc == got))
        # one rounding per instruction: c + sum_k a_k b_k exactly, rounded once
        acc = np.zeros((M, M), np.float32)
        for s in range(S):
            acc = (acc.astype(np.float64) + A[s].astype(np.float64) @ B[s].astype(np.float64)).astype(np.float32)
        res["one rounding per step"] = float(np.mean(acc == got))
        print(f"mfma f32 {shape}x{shape}x{kk} trial {trial}: " +
              ", ".join(f"{k} {v:.4f}" for k, v in res.items()), flush=True)
