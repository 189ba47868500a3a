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


def build_stamps(verbose=False, extra=(), suffix=""):
    """Diagnostic variant with in-kernel s_memtime stamps (-DGR_STAMPS) -> lib/libgr_amd_stamps*.so.
    Never loaded by the product path; used by scripts/stamps_rq.py only.  ``extra`` adds ablation
    macros (GR_ABL_*) for one-factor experiments."""
    os.makedirs(OBJDIR, exist_ok=True)
    out = os.path.join(LIBDIR, f"libgr_amd_stamps{suffix}.so")
    objs = []
    for src in sources():
        obj = os.path.join(OBJDIR, os.path.basename(src) + f".stamps{suffix}.o")
        cmd = [HIPCC] + (["-x", "hip"] if src.endswith(".cpp") else []) + CFLAGS + ["-DGR_STAMPS", *extra, "-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        objs.append(obj)
    subprocess.run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", out], check=True)
    return out


if __name__ == "__main__":
    import sys
    if "--abl" in sys.argv:   # diagnostic library with one GR_ABL_* macro (never loaded by the product)
        print(build_stamps(extra=[f"-D{sys.argv[sys.argv.index('--abl') + 1]}"], suffix="_abl"))
    elif "--stamps" in sys.argv:
        print(build_stamps())
        print(build_stamps(extra=["-DGR_ABL_NOW1"], suffix="_now1"))
        print(build_stamps(extra=["-DGR_ABL_NOX"], suffix="_nox"))
        print(build_stamps(extra=["-DGR_ABL_NOX", "-DGR_ABL_NOW1"], suffix="_noxw"))
        print(build_stamps(extra=["-DGR_ABL_W1COAL"], suffix="_w1coal"))
    else:
        print(build(verbose=True))
