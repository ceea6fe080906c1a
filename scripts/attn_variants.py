"""A/B timing of flash-attention forward kernel variants (the ``flags``
argument of dw_attn_fwd selects one; 0 = the default) on the same inputs,
interleaved so clock drift hits every variant alike.
    python scripts/attn_variants.py 8,1024,25,25,64 1,8192,32,8,128 --variants 0,1"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops import _hip  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    variants = [0, 1]
    if "--variants" in sys.argv:
        variants = [int(x) for x in sys.argv[sys.argv.index("--variants") + 1].split(",")]
        args = [a for a in args if a != sys.argv[sys.argv.index("--variants") + 1]]
    L = _hip.lib()
    for spec in args:
        B, S, H, HKV, D = map(int, spec.split(","))
        q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
        k = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16)
        v = torch.randn(B, S, HKV, D, device="cuda", dtype=torch.bfloat16)
        outs = {}

        def run(var):
            o = torch.empty_like(q)
            lse = torch.empty(B, H, S, device="cuda", dtype=torch.float32)
            _hip.check(L.dw_attn_fwd(_hip.ptr(q), _hip.ptr(k), _hip.ptr(v), _hip.ptr(o), _hip.ptr(lse), B, S, H, HKV,
                                     D, 1, float(D ** -0.5), var, _hip.stream()), "attn_fwd")
            return o

        for var in variants:
            outs[var] = run(var)
        ref = outs[variants[0]].float()
        times = {var: [] for var in variants}
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        for _rep in range(5):
            for var in variants:
                for _ in range(3):
                    run(var)
                ev[0].record()
                for _ in range(20):
                    run(var)
                ev[1].record()
                torch.cuda.synchronize()
                times[var].append(ev[0].elapsed_time(ev[1]) / 20)
        fl = 4 * B * H * S * S * D / 2
        for var in variants:
            t = sorted(times[var])[len(times[var]) // 2]
            err = (outs[var].float() - ref).abs().max().item()
            print(json.dumps({"shape": spec, "variant": var, "fwd_us": round(t * 1e3, 1),
                              "tflops": round(fl / t / 1e9, 1), "max_diff_vs_v0": err}), flush=True)


if __name__ == "__main__":
    main()
