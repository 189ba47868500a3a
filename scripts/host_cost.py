"""Host time per call of the reference's own call patterns and of their pieces:
``RQVAE.get_indices(x[64])`` (RQ-VAE/infer.py:93-95) and ``evaluate.rank_batch`` at 128 users
(SASRec/evaluate.py:21-32 at main.py's d 16), plus the Python / torch / ctypes primitives they use.
Prints one JSON line: median microseconds per call over ``--reps`` calls (no synchronisation)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gr_amd  # noqa: E402
from gr_amd import _lib as L, ops, synth  # noqa: E402
from gr_amd import evaluate as E  # noqa: E402


def med_us(fn, reps):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    ts = []
    for i in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if i % 64 == 63:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return float(np.median(ts)) * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    out = {}
    rq = synth.rqvae_model(3, 256, dev)
    x = synth.items(64, 77, dev)
    out["get_indices_b64"] = med_us(lambda: rq.get_indices(x), a.reps)
    b = rq.encode_binding()
    out["rq_encode_binding"] = med_us(lambda: ops.rq_encode(x, binding=b), a.reps)
    out["encode_binding_lookup"] = med_us(lambda: rq.encode_binding(), a.reps)
    out["packed_ptr"] = med_us(lambda: b.packed_ptr(), a.reps)
    # the C call alone, every argument prebuilt (its host cost = validation + the HIP launches)
    nb = b.workspace_bytes(64)
    wsp = torch.empty(nb, dtype=torch.uint8, device=dev)
    idx = torch.empty((64, 3), dtype=torch.int64, device=dev)
    args = (x.data_ptr(), 64, len(b.ws), b.dims_c, b.w_arr, b.b_arr, b.packed_ptr(), 3, b.ks_c, b.c_arr,
            idx.data_ptr(), None, None, None, wsp.data_ptr(), nb, L.stream_of(dev))
    fn = L.lib().gr_rq_encode_packed_f32
    out["c_call_rq_encode_packed"] = med_us(lambda: fn(*args), a.reps)
    items, n, d = 706, 20, 16
    p = synth.sasrec_params(d, n, 2, 1, 64, dev)
    sm = synth.sasrec_model(items, p, dev, seed=16)
    seqs = synth.sequences(128, n, items, 9000, dev)
    tg = torch.randint(1, items + 1, (128,), device=dev)
    out["rank_batch_b128"] = med_us(lambda: E.rank_batch(sm, seqs, tg), a.reps)
    out["last_hidden_b128"] = med_us(lambda: sm.last_hidden(seqs), a.reps)
    out["sasrec_binding_lookup"] = med_us(lambda: ops.sasrec_binding(sm), a.reps)
    # primitives
    out["torch_empty_small"] = med_us(lambda: torch.empty((64, 3), dtype=torch.int64, device=dev), a.reps)
    out["current_stream"] = med_us(lambda: torch.cuda.current_stream(dev).cuda_stream, a.reps)
    if hasattr(torch._C, "_cuda_getCurrentRawStream"):
        out["raw_stream"] = med_us(lambda: torch._C._cuda_getCurrentRawStream(0), a.reps)
    out["current_device"] = med_us(lambda: torch.cuda.current_device(), a.reps)

    def guard():
        with torch.cuda.device(dev):
            pass
    out["device_guard"] = med_us(guard, a.reps)
    out["is_capturing"] = med_us(lambda: torch.cuda.is_current_stream_capturing(), a.reps)
    lib = L.lib()
    out["ctypes_gr_version"] = med_us(lambda: lib.gr_version(), a.reps)
    out["data_ptr"] = med_us(lambda: x.data_ptr(), a.reps)
    out["c_void_p"] = med_us(lambda: L.ptr(x), a.reps)
    out["plus_one_kernel"] = med_us(lambda: tg + 1, a.reps)
    print(json.dumps({"host_us_median": out}), flush=True)


if __name__ == "__main__":
    main()
