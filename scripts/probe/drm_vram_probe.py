"""Does amdgpu's DRM fdinfo (drm-memory-vram) account a ROCm process's HIP
allocations?  Allocate 10 GiB through torch and compare."""
import glob
import os

import torch


def vram_kib(pid):
    tot = 0
    for fi in glob.glob(f"/proc/{pid}/fdinfo/*"):
        try:
            txt = open(fi).read()
        except OSError:
            continue
        for line in txt.splitlines():
            if line.startswith("drm-memory-vram:"):
                tot += int(line.split()[1])
    return tot


torch.cuda.init()
x = torch.empty(1, device="cuda")
torch.cuda.synchronize()
a = vram_kib(os.getpid())
y = torch.empty(10 << 30, dtype=torch.uint8, device="cuda")
y.fill_(1)
torch.cuda.synchronize()
b = vram_kib(os.getpid())
print(f"fdinfo vram before {a / 2**20:.2f} GiB after {b / 2**20:.2f} GiB (delta {(b - a) / 2**20:.2f}, expect 10)")
