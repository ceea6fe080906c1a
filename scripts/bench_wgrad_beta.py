"""Weight-gradient GEMM: accumulate (beta = 1, ``gb.addmm_``) vs overwrite
(beta = 0, ``torch.mm(out=gb)``) at the GPT2-1.5B shapes (8192 tokens).
Decides whether skipping the per-step gradient zeroing (first writer
overwrites) is worth it beyond the zero_ pass itself."""
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
    M = 8192
    tot = {"acc": 0.0, "over": 0.0}
    for N, K in [(4800, 1600), (1600, 1600), (6400, 1600), (1600, 6400)]:
        dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        g = torch.zeros(N, K, device="cuda", dtype=torch.bfloat16)
        acc = timeit(lambda: g.addmm_(dy.t(), x))
        over = timeit(lambda: torch.mm(dy.t(), x, out=g))
        tot["acc"] += acc
        tot["over"] += over
        print(json.dumps({"N": N, "K": K, "accumulate_us": round(acc, 1), "overwrite_us": round(over, 1),
                          "tflops_acc": round(2 * M * N * K / acc / 1e6, 1)}), flush=True)
    zero = torch.zeros(1557686400, device="cuda", dtype=torch.bfloat16)
    z = timeit(lambda: zero.zero_(), n=10)
    print(json.dumps({"per_layer_acc_us": round(tot["acc"], 1), "per_layer_over_us": round(tot["over"], 1),
                      "x48_saving_ms": round(48 * (tot["acc"] - tot["over"]) / 1000, 2),
                      "zero_grad_ms": round(z / 1000, 3)}), flush=True)


if __name__ == "__main__":
    main()
