"""Build a variant of the HIP kernel library with extra compiler flags for
A/B runs (load it with DWAMD_KERNELS_LIB_AB=<path>); the in-tree library is
untouched.
    python scripts/build_variant_lib.py gpurun_ab/libdw_kernels_noslp.so -fno-slp-vectorize"""
import glob
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd._native import build as b  # noqa: E402


def main():
    out, extra = os.path.abspath(sys.argv[1]), sys.argv[2:]
    odir = os.path.join(os.path.dirname(out), "obj_" + os.path.basename(out))
    os.makedirs(odir, exist_ok=True)
    objs = []
    procs = []
    for src in sorted(glob.glob(os.path.join(b.CSRC, "kernels", "*.hip"))):
        obj = os.path.join(odir, os.path.basename(src) + ".o")
        cmd = [b._hipcc(), f"--offload-arch={b.ARCH}", "-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5",
               "-munsafe-fp-atomics", "-ffp-contract=fast", "-mllvm", "-amdgpu-mfma-vgpr-form",
               "-Wno-unused-result", "-I", os.path.join(b.CSRC, "kernels")] + b.FILE_FLAGS.get(
                   os.path.basename(src), []) + extra + ["-c", src, "-o", obj]
        procs.append(subprocess.Popen(cmd))
        objs.append(obj)
    assert all(p.wait() == 0 for p in procs)
    subprocess.check_call([b._hipcc(), f"--offload-arch={b.ARCH}", "-shared", "-fPIC", "-o", out] + objs
                          + ["-lhipblaslt"])
    print(out)


if __name__ == "__main__":
    main()
