"""Snapshot-copy bandwidth (HBM -> HBM, the flash-checkpoint training pause)
for the multi-copy kernel variants, the grid cap and the descriptor chunk,
against one hipMemcpy D2D.  GPT2-1.5B flat state size (21.8 GB) by default.
One JSON line per case; GB/s = bytes copied / s (HBM traffic is 2x)."""

import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd._native import kernels  # noqa: E402

L = kernels(required=True)
n = int(float(os.environ.get("COPY_GB", "21.8")) * 1e9) // 4096 * 4096
src = torch.empty(n, dtype=torch.uint8, device="cuda")
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
src.view(torch.int32)[: n // 4].random_()


def descs(chunk):
    o = np.arange(0, n, chunk, dtype=np.uint64)
    a = np.empty((o.size, 3), dtype=np.uint64)
    a[:, 0] = o + np.uint64(src.data_ptr())
    a[:, 1] = o + np.uint64(dst.data_ptr())
    a[:, 2] = np.minimum(np.uint64(chunk), np.uint64(n) - o)
    return torch.from_numpy(a.view(np.int64)).cuda()


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
t = timed(lambda: dst.copy_(src))
print(json.dumps({"case": "hipMemcpy D2D", "ms": round(t * 1e3, 3), "gbps": round(n / t / 1e9, 1)}), flush=True)
for chunk_mb in (1, 4):
    d = descs(chunk_mb << 20)
    for variant in (0, 1, 2, 3):
        for blocks in (1024, 2048, 4096):
            t = timed(lambda: L.dw_multi_copy_variant(ctypes.c_void_p(d.data_ptr()), d.shape[0], variant, blocks, s))
            print(json.dumps({"case": "multi_copy", "variant": variant, "blocks": blocks, "chunk_mb": chunk_mb,
                              "ms": round(t * 1e3, 3), "gbps": round(n / t / 1e9, 1)}), flush=True)
assert torch.equal(dst[:1 << 20], src[:1 << 20]) and torch.equal(dst[-(1 << 20):], src[-(1 << 20):])
