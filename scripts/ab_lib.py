"""Device-time A/B of two builds of libgr_amd.so on the RQ encode kernels (gr_rq_mlp_f32 = the
encoder, gr_rq_quantize_f32 = the quantizer), each call graph-captured 20 times and replayed, on
the C2 bench workload.  Both libraries are loaded side by side (RTLD_LOCAL); same inputs.

    python scripts/ab_lib.py lib/libgr_amd_r02.so lib/libgr_amd.so [--n 100000] [--L 3 --K 256]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib as L, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--n", type=int, default=100_000)
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
ap.add_argument("--calls", type=int, default=0, help="just issue this many plain calls per library (for rocprofv3)")
ap.add_argument("--what", default="rq", help="rq: encoder + quantizer; topk: gr_score_topk_f32 (d 128, 512 users)")
ap.add_argument("--rows", type=int, default=1_000_001, help="topk: catalog rows")
a = ap.parse_args()
dev = torch.device("cuda:0")
def cur():
    """The stream the caller is on NOW (a graph capture runs on a side stream)."""
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def graph_us(fn, calls=20, reps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    for _ in range(30):
        g.replay()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * calls) * 1e3


if a.what == "topk":   # fused score + top-10 + strict counts over a catalog (SASRec C5 / shard)
    B, d, k = 512, 128, 10
    g = torch.Generator(device=dev).manual_seed(0)
    h = torch.randn(B, d, generator=g, device=dev) * 0.1
    table = torch.randn(a.rows, d, generator=g, device=dev) * 0.1
    thr = torch.randn(B, generator=g, device=dev) * 0.1
    ref = None
    for path in a.libs:
        lib = ctypes.CDLL(os.path.abspath(path))
        lib.gr_score_topk_workspace_bytes.restype = ctypes.c_size_t
        lib.gr_score_topk_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32]
        nb = lib.gr_score_topk_workspace_bytes(B, d, a.rows, k)
        ws = torch.empty(nb, dtype=torch.uint8, device=dev)
        vals = torch.empty((B, k), device=dev)
        ids = torch.empty((B, k), dtype=torch.int64, device=dev)
        cnt = torch.empty(B, dtype=torch.int64, device=dev)
        vp = ctypes.c_void_p
        fn = lambda: lib.gr_score_topk_f32(vp(h.data_ptr()), ctypes.c_int64(B), d, vp(table.data_ptr()),  # noqa
                                           ctypes.c_int64(a.rows), ctypes.c_int64(0), 1, k, vp(thr.data_ptr()),
                                           vp(cnt.data_ptr()), vp(vals.data_ptr()), vp(ids.data_ptr()),
                                           vp(ws.data_ptr()), ctypes.c_size_t(nb), cur())
        assert fn() == 0
        torch.cuda.synchronize()
        same = "" if ref is None else f"  same results: {torch.equal(ids, ref[0]) and torch.equal(cnt, ref[1])}"
        ref = (ids.clone(), cnt.clone()) if ref is None else ref
        if a.calls:
            for _ in range(a.calls):
                fn()
            torch.cuda.synchronize()
            continue
        print(f"{os.path.basename(path):24s} topk B={B} d={d} rows={a.rows}: {graph_us(fn, calls=5):9.2f} us{same}",
              flush=True)
    sys.exit(0)
m = synth.rqvae_model(a.L, a.K, dev)
b = m.encode_binding()
x = synth.items(a.n, 1000, dev)


ref_idx = None
for path in a.libs:
    lib = ctypes.CDLL(os.path.abspath(path))
    lib.gr_rq_mlp_workspace_bytes.restype = ctypes.c_size_t
    lib.gr_rq_mlp_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p]
    n = a.n
    dims = L.i32_array(b.dims)
    nb = lib.gr_rq_mlp_workspace_bytes(n, len(b.ws), dims)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    z = torch.empty((n, b.dims[-1]), device=dev)
    idx = torch.empty((n, len(b.cbs)), dtype=torch.int64, device=dev)
    wa, ba, ca, ks = L.ptr_array(b.ws), L.ptr_array(b.bs), L.ptr_array(b.cbs), L.i32_array(b.Ks)
    mlp = lambda: lib.gr_rq_mlp_f32(ctypes.c_void_p(x.data_ptr()), ctypes.c_int64(n), len(b.ws), dims, wa, ba,  # noqa
                                    ctypes.c_void_p(z.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                    ctypes.c_size_t(nb), cur())
    quant = lambda: lib.gr_rq_quantize_f32(ctypes.c_void_p(z.data_ptr()), ctypes.c_int64(n), b.dims[-1],  # noqa
                                           len(b.cbs), ks, ca, None, ctypes.c_void_p(idx.data_ptr()), None, None, cur())
    assert mlp() == 0 and quant() == 0
    torch.cuda.synchronize()
    if a.calls:
        for _ in range(a.calls):
            mlp()
            quant()
        torch.cuda.synchronize()
        continue
    same = "" if ref_idx is None else f"  rows differing from the first library: {(idx != ref_idx).any(1).sum().item()}"
    ref_idx = idx.clone() if ref_idx is None else ref_idx
    print(f"{os.path.basename(path):24s} n={n} L={a.L} K={a.K}: encoder {graph_us(mlp):8.2f} us  "
          f"quantize {graph_us(quant):8.2f} us{same}", flush=True)
