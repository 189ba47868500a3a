"""Per-workgroup phase timestamps of the one-launch encode (gr_rq_encode_stamps): when each
workgroup finished its encoder tiles, staged the codebooks and finished quantizing, and how many
4-tile groups it quantized.  Times in microseconds from the earliest workgroup start.

    python scripts/stamps_encq.py [--n 100000] [--L 3 --K 256]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from gr_amd import _lib as L, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=100_000)
ap.add_argument("--L", type=int, default=3)
ap.add_argument("--K", type=int, default=256)
a = ap.parse_args()
dev = torch.device("cuda:0")
rq = synth.rqvae_model(a.L, a.K, dev)
x = synth.items(a.n, 1000, dev)
cus = torch.cuda.get_device_properties(0).multi_processor_count
st = torch.zeros(8 * cus, dtype=torch.int64, device=dev)
lib = L.lib()
lib.gr_rq_encode_stamps.argtypes = [ctypes.c_void_p]
for _ in range(20):
    rq.get_indices(x)
torch.cuda.synchronize()
lib.gr_rq_encode_stamps(ctypes.c_void_p(st.data_ptr()))
for rep in range(3):
    st.zero_()
    rq.get_indices(x)
    torch.cuda.synchronize()
    s = st.view(-1, 8).cpu().double()
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    us = lambda v: (v - t0) / 100.0  # noqa: E731
    start, enc, staged, end = us(s[:, 0]), us(s[:, 1]), us(s[:, 2]), us(s[:, 3])
    print(f"rep {rep}: {len(s)} workgroups; kernel span {end.max():.1f} us", flush=True)
    for tiles in sorted(set(s[:, 6].long().tolist())):
        m = s[:, 6] == tiles
        print(f"  {int(m.sum()):3d} WGs with {tiles:3d} encoder tiles: start {start[m].min():6.1f}-{start[m].max():6.1f}"
              f"  encoder done {enc[m].min():6.1f}-{enc[m].max():6.1f} (mean {enc[m].mean():6.1f})"
              f"  staged +{(staged[m] - enc[m]).mean():5.1f}  end {end[m].min():6.1f}-{end[m].max():6.1f}"
              f"  groups {s[m, 4].mean():4.2f} (max {int(s[m, 4].max())})  polls {s[m, 5].mean():7.1f}"
              + (f"  last (odd) pass {(enc[m] - us(s[m, 7])).mean():5.1f}" if s[m, 7].min() > 0 else ""), flush=True)
lib.gr_rq_encode_stamps(None)
