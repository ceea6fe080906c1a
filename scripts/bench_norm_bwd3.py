"""Norm backward as the GPT2-1.5B step calls it (LayerNorm, H = 1600, rows =
B*S = 8192, residual gradient fused in, dx column sums for the folded Linear
bias): dw_norm_bwd3 timed alone, plus a bitwise check against the library
named by DWAMD_KERNELS_LIB_REF (when set).
    DWAMD_KERNELS_LIB_AB=gpurun_ab/libdw_kernels_w2.so python scripts/bench_norm_bwd3.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dlrover_wuqiong_amd.ops import _hip  # noqa: E402


def run(R=8192, H=1600, iters=100, rms=False, with_dsum=True):
    g = torch.Generator(device="cpu").manual_seed(0)
    dev = "cuda"
    x = torch.randn(R, H, generator=g).to(dev, torch.bfloat16)
    dy = torch.randn(R, H, generator=g).to(dev, torch.bfloat16)
    dres = torch.randn(R, H, generator=g).to(dev, torch.bfloat16)
    w = torch.randn(H, generator=g).to(dev, torch.bfloat16)
    if rms:  # RMSNorm (Llama): no mean, rstd of the mean square
        mean = torch.zeros(R, device=dev)
        rstd = (x.float().pow(2).mean(-1) + 1e-5).rsqrt().contiguous()
    else:
        mean = x.float().mean(-1).contiguous()
        rstd = (x.float().var(-1, unbiased=False) + 1e-5).rsqrt().contiguous()
    dx = torch.empty_like(x)
    dgamma = torch.zeros(H, device=dev, dtype=torch.float32)
    dbeta = torch.zeros(H, device=dev, dtype=torch.float32)
    dsum = torch.zeros(H, device=dev, dtype=torch.float32)
    ws = _hip.zeroed_workspace(3 * H + max((H + 511) // 512, (3 * H + 255) // 256), x.device)
    nparts = min(512, (R + 1) // 2) * 3 * H  # as ops/norm.py
    part = torch.empty(nparts, device=dev, dtype=torch.float32)
    done = ctypes.c_int(0)

    def call():
        _hip.check(_hip.lib().dw_norm_bwd3(_hip.ptr(dy), _hip.ptr(x), _hip.ptr(w), _hip.ptr(mean), _hip.ptr(rstd),
                                           _hip.ptr(dres), _hip.ptr(dx), _hip.ptr(dgamma), _hip.ptr(dbeta),
                                           _hip.ptr(ws), _hip.ptr(part), nparts, R, H, int(rms), 1, 2,
                                           _hip.ptr(dsum if with_dsum else None),
                                           ctypes.byref(done), _hip.stream(), None), "norm_bwd3")

    for _ in range(5):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = 1000 * e0.elapsed_time(e1) / iters
    # reference (fp32 torch): dx = rstd*(dy*w - mean(dy*w) - xhat*mean(dy*w*xhat)) + dres
    xh = (x.float() - mean[:, None]) * rstd[:, None]
    gdy = dy.float() * w.float()
    m1 = 0.0 if rms else gdy.mean(-1, keepdim=True)
    ref = rstd[:, None] * (gdy - m1 - xh * (gdy * xh).mean(-1, keepdim=True)) + dres.float()
    err = float((dx.float() - ref).abs().max())
    dg_ref = (dy.float() * xh).sum(0)
    dg_err = float((dgamma - dg_ref).abs().max() / dg_ref.abs().max())
    nbytes = 4 * R * H * 2  # x, dy, dres read + dx written
    return {"R": R, "H": H, "rms": rms, "us": round(us, 2), "tbs": round(nbytes / (us * 1e-6) / 1e12, 2), "dx_maxerr": err,
            "dgamma_relerr": dg_err, "dsum_done": done.value,
            "lib": os.path.basename(os.environ.get("DWAMD_KERNELS_LIB_AB", "")) or "in-tree"}


if __name__ == "__main__":
    if "--llama" in sys.argv:  # Llama-3-8B's call: RMSNorm, H = 4096, 4096 rows, no folded bias
        for R in (4096, 8192):
            print(json.dumps(run(R, 4096, rms=True, with_dsum=False)), flush=True)
    else:
        for R in (8192, 16384):
            print(json.dumps(run(R)), flush=True)
