"""GPT2-1.5B attention-projection weight gradient dW[1600,1600] = dy^T x
over 8192 tokens: hipBLASLt runs it at ~0.46 PF in the step (39 output
tiles of 256x256 for 256 CUs).  Times the library GEMM against split-K
forms: K cut into S chunks as one batched GEMM with fp32 partials
(``out_dtype`` when this torch has it) plus a sum."""
import json

import torch


def timeit(fn, n=30):
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
    M, N, K = 8192, 1600, 1600
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    gw = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
    ref = dy.float().t() @ x.float()
    fl = 2 * M * N * K

    def rep(name, us, out):
        err = float((out.float() - ref).abs().max() / ref.abs().max())
        print(json.dumps({"variant": name, "us": round(us, 1), "tflops": round(fl / us / 1e6, 1), "rel_err": err}),
              flush=True)

    rep("mm_out_beta0", timeit(lambda: torch.mm(dy.t(), x, out=gw)), gw)
    gw.zero_()
    rep("addmm_beta1", timeit(lambda: gw.addmm_(dy.t(), x)), (gw.zero_().addmm_(dy.t(), x)))
    for S in (2, 4, 8):
        a = dy.view(S, M // S, N).transpose(1, 2)
        b = x.view(S, M // S, K)
        try:
            part = torch.empty(S, N, K, device="cuda", dtype=torch.float32)

            def f32():
                torch.bmm(a, b, out_dtype=torch.float32, out=part)
                torch.sum(part, 0, out=gw)

            us = timeit(f32)
            rep(f"splitk{S}_fp32", us, gw)
        except Exception as e:  # no out_dtype on this torch
            print(json.dumps({"variant": f"splitk{S}_fp32", "error": str(e)[:120]}), flush=True)
        pb = torch.empty(S, N, K, device="cuda", dtype=torch.bfloat16)

        def bf():
            torch.bmm(a, b, out=pb)
            torch.sum(pb, 0, out=gw)

        us = timeit(bf)
        rep(f"splitk{S}_bf16partials", us, gw)


if __name__ == "__main__":
    main()
