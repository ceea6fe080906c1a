"""Column-reduction kernels (bias gradients) on the GPT2-1.5B shapes:
colsum (dbias of a [8192, C] bf16 gradient) and the fused GELU backward +
dbias.  One JSON line per shape with the achieved HBM GB/s; run once per
DWAMD_COLRED_BLOCKS value for the grid-size A/B."""

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops import _hip  # noqa: E402
from dlrover_wuqiong_amd.ops.activation import colsum  # noqa: E402


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e-3


R = 8192
blocks = os.environ.get("DWAMD_COLRED_BLOCKS", "1024")
for C in (1600, 4800, 6400):
    dy = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
    out = torch.zeros(C, device="cuda", dtype=torch.float32)
    t = timed(lambda: colsum(dy, out=out, accumulate=False))
    ref = dy.float().sum(0)
    err = float((out - ref).abs().max() / ref.abs().max())
    print(json.dumps({"op": "colsum", "blocks": blocks, "R": R, "C": C, "us": round(t * 1e6, 1),
                      "gbps": round(R * C * 2 / t / 1e9, 1), "rel_err": err}), flush=True)
    if C == 6400:
        pre = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
        dx = torch.empty_like(dy)
        ws = _hip.zeroed_workspace(C + (C + 511) // 512, dy.device)
        L = _hip.lib()

        def gb():
            _hip.check(L.dw_gelu_bwd_dbias(_hip.ptr(dy), _hip.ptr(pre), _hip.ptr(dx), R, C, _hip.ptr(ws),
                                           _hip.ptr(out), 1, 0, _hip.stream(), None), "gelu_bwd_dbias")
        t = timed(gb)
        print(json.dumps({"op": "gelu_bwd_dbias", "blocks": blocks, "R": R, "C": C, "us": round(t * 1e6, 1),
                          "gbps": round(3 * R * C * 2 / t / 1e9, 1)}), flush=True)
