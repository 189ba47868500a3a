"""Per-phase cycle shares of the fused RQ kernel from the diagnostic stamps build
(lib/libgr_amd_stamps.so, build.py --stamps).  Read the SHARES, not the absolute time: the stamps
fence the schedule (cdna guide §7, In-kernel stamps)."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gr_amd import _lib  # noqa: E402

VARIANT = os.environ.get("GR_STAMPS_VARIANT", "")
_lib.LIB_PATH = os.path.join(os.path.dirname(_lib.LIB_PATH), f"libgr_amd_stamps{VARIANT}.so")
from gr_amd import synth  # noqa: E402

L = int(sys.argv[1]) if len(sys.argv) > 1 else 3
K = int(sys.argv[2]) if len(sys.argv) > 2 else 256
dev = torch.device("cuda:0")
m = synth.rqvae_model(L, K, dev)
x = synth.items(100_000, 7, dev)
lib = _lib.lib()
if os.environ.get("GR_ENC_W8") is not None:   # 8-wave (1) or 4-wave (0) fused encoder
    _lib.set_option("rq_enc_w8", int(os.environ["GR_ENC_W8"]))
lib.gr_debug_rq_stamps.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 10)()
m.get_indices(x)
torch.cuda.synchronize()
lib.gr_debug_rq_stamps(buf)
REPS = 5
for _ in range(REPS):
    m.get_indices(x)
torch.cuda.synchronize()
lib.gr_debug_rq_stamps(buf)
names = ["L1", "h1 store", "L2", "L3", "z store"]
tot = sum(buf[i] for i in range(5))
print(f"[{VARIANT or 'base'}] L={L} K={K} tiles={buf[5]}  cycles/tile (wave 0): {tot / max(buf[5], 1):.0f}")
mf = {"L1": 768, "h1 store": 0, "L2": 128, "L3": 16, "z store": 0}
for i, nm in enumerate(names):
    per_tile = buf[i] / max(buf[5], 1)
    print(f"  {nm:9s} {100 * buf[i] / tot:5.1f} %   {per_tile:9.0f} cyc/tile   MFMA floor {mf[nm] * 64:7.0f}")
if buf[7]:
    print(f"  effective clock {100e6 * buf[6] / buf[7] / 1e9:.3f} GHz (sum over workgroups); "
          f"longest workgroup {buf[8]} cyc = {buf[9] / 100:.1f} us (max over {REPS} launches)")
