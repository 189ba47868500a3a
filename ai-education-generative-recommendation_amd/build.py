"""Build libgr_amd.so (the C-ABI HIP library, include/gr_amd.h) in-tree for gfx950.

    python -m ... / __graft_entry__.build()  ->  <package>/lib/libgr_amd.so

Plain ``hipcc`` per translation unit (parallel), then one shared link.  The result stays inside the
package directory so it travels with the repository snapshot to the GPU box.
"""
import concurrent.futures as cf
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "lib")
OBJDIR = os.path.join(ROOT, "build", "obj")
LIB = os.path.join(LIBDIR, "libgr_amd.so")
ARCH = "gfx950"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
          "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function"]


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _deps():
    hdrs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    hdrs.append(os.path.join(ROOT, "include", "gr_amd.h"))
    return max(os.path.getmtime(h) for h in hdrs)


def _compile(src, dep_mtime, verbose):
    obj = os.path.join(OBJDIR, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), dep_mtime):
        return obj
    cmd = [HIPCC, *CFLAGS, "-c", src, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC, "-x", "hip", *CFLAGS, "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return obj


def build(verbose=False, force=False):
    """Compile every HIP source for gfx950 and link ``lib/libgr_amd.so``; returns the library path."""
    os.makedirs(OBJDIR, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    dep = _deps()
    if force:
        for f in os.listdir(OBJDIR):
            os.remove(os.path.join(OBJDIR, f))
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, dep, verbose), srcs))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", LIB + ".tmp"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB


if __name__ == "__main__":
    print(build(verbose=True))
