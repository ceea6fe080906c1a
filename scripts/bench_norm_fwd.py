"""Norm forward micro-benchmark: fused add + LayerNorm / RMSNorm and plain
norm at the GPT2-1.5B / Llama shapes, and the MLP's GELU pass.  Prints one
JSON line per shape with the HBM rate (x, res read; h, y written for the add
form).  profiles/r4/norm_fwd_gelu_ab.jsonl holds the round-4 A/B of the
grid-stride norm / unrolled GELU variants it was written for (both equal to
the kept kernels, since removed)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dlrover_wuqiong_amd.ops.norm import add_layer_norm, add_rms_norm, layer_norm  # noqa: E402


def timeit(fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return 1000 * e0.elapsed_time(e1) / n


def main():
    var = os.environ.get("DWAMD_NORM_FWD_BLOCKS", "default")
    with torch.no_grad():
        for R, H, kind in [(8192, 1600, "add_ln"), (16384, 1600, "add_ln"), (8192, 1600, "ln"),
                           (16384, 4096, "add_rms"), (8192, 1024, "add_rms")]:
            x = torch.randn(R, H, device="cuda", dtype=torch.bfloat16)
            r = torch.randn(R, H, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(H, device="cuda", dtype=torch.bfloat16)
            b = torch.randn(H, device="cuda", dtype=torch.bfloat16)
            if kind == "add_ln":
                fn, nb = (lambda: add_layer_norm(x, r, w, b)), 4
                yr, hr = torch.nn.functional.layer_norm((x.float() + r.float()), (H,), w.float(), b.float()), None
            elif kind == "add_rms":
                fn, nb = (lambda: add_rms_norm(x, r, w)), 4
                yr = None
            else:
                fn, nb = (lambda: layer_norm(x, w, b)), 2
                yr = torch.nn.functional.layer_norm(x.float(), (H,), w.float(), b.float())
            out = fn()
            y = out[0] if isinstance(out, tuple) else out
            err = float((y.float() - yr).abs().max()) if yr is not None else None
            us = timeit(fn)
            print(json.dumps({"kind": kind, "R": R, "H": H, "blocks": var, "us": round(us, 1),
                              "hbm_tbs": round(nb * R * H * 2 / (us * 1e-6) / 1e12, 2), "max_err": err}), flush=True)


def gelu_main():
    """GELU pass of the fused MLP (``DWAMD_GELU_UNROLL``: 1 = plain loop)."""
    from dlrover_wuqiong_amd.ops import _hip

    for R, C in [(8192, 6400), (16384, 6400)]:
        x = torch.randn(R, C, device="cuda", dtype=torch.bfloat16)
        y = torch.empty_like(x)

        def fn():
            _hip.check(_hip.lib().dw_bias_gelu_fwd(_hip.ptr(x), None, _hip.ptr(y), None, x.numel(), C,
                                                   _hip.stream()), "gelu")

        fn()
        err = float((y.float() - torch.nn.functional.gelu(x.float(), approximate="tanh")).abs().max())
        us = timeit(fn)
        print(json.dumps({"kind": "gelu", "R": R, "C": C, "unroll": os.environ.get("DWAMD_GELU_UNROLL", "default"),
                          "us": round(us, 1), "hbm_tbs": round(2 * R * C * 2 / (us * 1e-6) / 1e12, 2),
                          "max_err": err}), flush=True)


if __name__ == "__main__":
    main()
    gelu_main()
