"""In-tree build of the native libraries (gfx950 only).

``python -m dlrover_wuqiong_amd._native.build`` builds both libraries.
Every ``csrc/kernels/*.hip`` translation unit is compiled separately (in
parallel) with ``hipcc --offload-arch=gfx950`` and linked into
``libdw_kernels.so``; ``csrc/runtime/*.cpp`` is compiled with the host
compiler into ``libdw_runtime.so``.
"""

import glob
import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
BUILD_DIR = os.path.join(HERE, "_build")
ARCH = os.environ.get("DWAMD_OFFLOAD_ARCH", "gfx950")


def runtime_lib_path():
    return os.path.join(HERE, "libdw_runtime.so")


def kernels_lib_path():
    return os.path.join(HERE, "libdw_kernels.so")


def sources_for(which):
    if which == "runtime":
        return sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp"))) + sorted(
            glob.glob(os.path.join(CSRC, "runtime", "*.h")))
    # this file too: its compiler flags are part of what the library is
    return sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip"))) + sorted(
        glob.glob(os.path.join(CSRC, "kernels", "*.h"))) + [os.path.abspath(__file__)]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _atomic_replace(tmp, dst):
    os.replace(tmp, dst)


def sources_digest(which) -> str:
    """Content hash of a library's sources: a copied tree (tar, rsync) keeps
    the library fresh even when file times change."""
    import hashlib

    h = hashlib.sha256()
    for s in sources_for(which):
        h.update(os.path.basename(s).encode())
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _write_digest(lib_path, which):
    with open(lib_path + ".srcsha.tmp", "w") as f:
        f.write(sources_digest(which))
    os.replace(lib_path + ".srcsha.tmp", lib_path + ".srcsha")


class _BuildLock:
    """One builder per tree: concurrent processes (workers + standbys that
    find the library stale) wait instead of racing on the same objects."""

    def __init__(self):
        os.makedirs(BUILD_DIR, exist_ok=True)
        self.path = os.path.join(BUILD_DIR, ".lock")

    def __enter__(self):
        import fcntl

        self.f = open(self.path, "w")
        fcntl.flock(self.f, fcntl.LOCK_EX)
        return self

    def __exit__(self, *a):
        import fcntl

        fcntl.flock(self.f, fcntl.LOCK_UN)
        self.f.close()


def build_runtime(verbose=False):
    with _BuildLock():
        return _build_runtime(verbose)


def _build_runtime(verbose=False):
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = [s for s in sources_for("runtime") if s.endswith(".cpp")]
    out = runtime_lib_path()
    tmp = out + f".tmp{os.getpid()}"
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-msse4.2", "-pthread",
           "-Wall", "-Wno-unused-result", "-o", tmp] + srcs + ["-lrt"]
    o = _run(cmd)
    if verbose and o:
        print(o)
    _atomic_replace(tmp, out)
    _write_digest(out, "runtime")
    return out


# Per-file extra flags.  Attention: no SLP vectorisation -- the vectoriser
# packs adjacent f32 multiplies / adds into v_pk_*_f32, which cost more than
# two scalar ops when issued beside MFMAs (MI355X_MICROARCH 'price of one
# filler'); measured GPT2-shape backward 368 -> 379 TF/s, D=128 within +-1 %
# (profiles/r3/attn_bench_{slp,noslp}.jsonl).
FILE_FLAGS = {"attn_bwd.hip": ["-fno-slp-vectorize"], "attn_fwd.hip": ["-fno-slp-vectorize"],
              "attn_bwd_dq2.hip": ["-fno-slp-vectorize"], "attn_fwd2.hip": ["-fno-slp-vectorize"]}


def _compile_hip(src):
    obj = os.path.join(BUILD_DIR, os.path.basename(src) + ".o")
    deps = [src, os.path.abspath(__file__)] + glob.glob(os.path.join(CSRC, "kernels", "*.h"))
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
           "-mcode-object-version=5", "-munsafe-fp-atomics", "-ffp-contract=fast",
           # MFMA accumulators in arch VGPRs: with a 512-register budget (one
           # wave per SIMD allowed by the launch bounds) the default AGPR form
           # costs v_accvgpr_read/write copies around every softmax
           # (attention D=64: 176 extra VALU ops per 64-key tile)
           "-mllvm", "-amdgpu-mfma-vgpr-form",
           "-Wno-unused-result", "-I", os.path.join(CSRC, "kernels")] + FILE_FLAGS.get(os.path.basename(src), []) + [
           "-c", src, "-o", obj + f".tmp{os.getpid()}"]
    _run(cmd)
    os.replace(obj + f".tmp{os.getpid()}", obj)
    return obj


def build_kernels(verbose=False, jobs=None):
    with _BuildLock():
        return _build_kernels(verbose, jobs)


def _build_kernels(verbose=False, jobs=None):
    os.makedirs(BUILD_DIR, exist_ok=True)
    srcs = [s for s in sources_for("kernels") if s.endswith(".hip")]
    jobs = jobs or min(8, max(1, len(srcs)))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile_hip, srcs))
    out = kernels_lib_path()
    tmp = out + f".tmp{os.getpid()}"
    # hipBLASLt for the epilogue-fused GEMMs (gemm_epilogue.hip)
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs + ["-lhipblaslt"]
    o = _run(cmd)
    if verbose and o:
        print(o)
    _atomic_replace(tmp, out)
    _write_digest(out, "kernels")
    return out


def build_all(verbose=True):
    r = build_runtime(verbose)
    k = build_kernels(verbose)
    if verbose:
        print(f"built {r}\nbuilt {k}")
    return r, k


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which == "runtime":
        build_runtime(True)
    elif which == "kernels":
        build_kernels(True)
    else:
        build_all(True)
