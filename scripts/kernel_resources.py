"""Per-kernel register / scratch usage of a .hip file for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel:
    python scripts/kernel_resources.py dlrover_wuqiong_amd/csrc/kernels/attn_fwd.hip [filter]
extra compiler flags via KRES_FLAGS (e.g. "-mllvm -amdgpu-mfma-vgpr-form")."""
import os
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    extra = os.environ.get("KRES_FLAGS", "").split()
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o",
                        "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra, capture_output=True, text=True)
    cur, rows = None, []
    for ln in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill|"
                      r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", ln)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for c in rows:
        if flt in c["name"]:
            print(f"{c['name'][:90]:90s} vgpr={c.get('VGPRs')} agpr={c.get('AGPRs')} "
                  f"scratch={c.get('ScratchSize [bytes/lane]')} vspill={c.get('VGPRs Spill')} "
                  f"occ={c.get('Occupancy [waves/SIMD]')}")
    if r.returncode:
        print(r.stderr[-3000:])


if __name__ == "__main__":
    main()
