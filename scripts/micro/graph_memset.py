"""Do captured memset nodes keep stream order when one graph is replayed back to back?

Graph = [hipMemsetAsync(buf, 0)] -> [buf += 1] -> [acc += buf] (torch kernels), captured with
torch.cuda.graph.  Replayed N times with no host synchronisation, every element of acc must be N;
an element above N means a replay's memset did not clear buf before that replay's kernels read it.
The same graph with the memset replaced by a kernel (buf.zero_() -> fill kernel) is the control.
Wrong values only -- nothing here can fault."""
import ctypes
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
dev = torch.device("cuda:0")


def run(kind, numel, reps, inflight_sync_every=0):
    buf = torch.zeros(numel, dtype=torch.float32, device=dev)
    acc = torch.zeros(numel, dtype=torch.float32, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        buf.add_(1)
        acc.add_(buf)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        if kind == "memset":
            st = torch.cuda.current_stream().cuda_stream
            assert hip.hipMemsetAsync(ctypes.c_void_p(buf.data_ptr()), 0, buf.numel() * 4, ctypes.c_void_p(st)) == 0
        else:
            buf.fill_(0.0)
        buf.add_(1)
        acc.add_(buf)
    acc.zero_()
    torch.cuda.synchronize()
    for i in range(reps):
        g.replay()
        if inflight_sync_every and (i + 1) % inflight_sync_every == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    bad = (acc != reps).sum().item()
    print(f"{kind:7s} numel {numel:>10d} replays {reps:5d} sync every {inflight_sync_every or 'never':>5}: "
          f"elements != replays: {bad} (max {acc.max().item():.0f})", flush=True)
    return bad


for numel in (256, 65536, 16 << 20):
    for kind in ("memset", "kernel"):
        run(kind, numel, 400)
        run(kind, numel, 400, inflight_sync_every=1)
sys.exit(0)
