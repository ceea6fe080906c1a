"""Grouped GEMM TF/s on Mixtral-8x7B expert shapes (E=8, H=4096, F=14336,
16384 routed rows = 8192 tokens x top-2) vs a per-expert loop of
torch.nn.functional.linear (hipBLASLt).  Prints one JSON line."""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops.grouped_gemm import MODE_NN, MODE_NT, MODE_TN, _launch, offsets_from_counts  # noqa


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def run(E, H, Fd, T, name):
    torch.manual_seed(0)
    g = torch.Generator().manual_seed(0)
    probs = torch.rand(E, generator=g) + 0.5
    counts = (probs / probs.sum() * T).long()
    counts[-1] += T - counts.sum()
    dev = "cuda"
    x = torch.randn(T, H, device=dev, dtype=torch.bfloat16)
    w = torch.randn(E, Fd, H, device=dev, dtype=torch.bfloat16) * 0.02
    dy = torch.randn(T, Fd, device=dev, dtype=torch.bfloat16)
    counts_d = counts.to(dev)
    offs = offsets_from_counts(counts_d, dev)
    y = torch.empty(T, Fd, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(T, H, device=dev, dtype=torch.bfloat16)
    dw = torch.empty_like(w)
    flops = 2 * T * H * Fd
    res = {"metric": f"grouped GEMM TF/s ({name}: E={E}, H={H}, F={Fd}, {T} rows)",
           "rows_per_expert_mean": T // E}
    res["nt_fwd_tfs"] = round(flops / timeit(lambda: _launch(MODE_NT, x, w, y, offs, E, T, 0, Fd, H, H, H, Fd,
                                                                 Fd * H, 0)) / 1e12, 1)
    res["nn_dgrad_tfs"] = round(flops / timeit(lambda: _launch(MODE_NN, dy, w, dx, offs, E, T, 0, H, Fd, Fd, H, H,
                                                                   Fd * H, 0)) / 1e12, 1)
    res["tn_wgrad_tfs"] = round(flops / timeit(lambda: _launch(MODE_TN, dy, x, dw, offs, E, T, Fd, H, 0, Fd, H, H, 0,
                                                                   Fd * H)) / 1e12, 1)
    cl = counts.tolist()

    def loop_fwd():
        o = 0
        cl = counts_d.tolist()  # the device->host sync a per-expert loop needs
        for e in range(E):
            F.linear(x[o:o + cl[e]], w[e])
            o += cl[e]

    res["per_expert_loop_fwd_tfs"] = round(flops / timeit(loop_fwd) / 1e12, 1)
    # correctness spot check vs the loop
    _launch(MODE_NT, x, w, y, offs, E, T, 0, Fd, H, H, H, Fd, Fd * H, 0)
    o = cl[0]
    ref = F.linear(x[o:o + cl[1]], w[1])
    res["max_rel_err_expert1"] = float(((y[o:o + cl[1]].float() - ref.float()).norm() / ref.float().norm()))
    print(json.dumps(res), flush=True)


def main():
    run(8, 4096, 14336, 16384, "Mixtral-8x7B expert w1")
    run(64, 2048, 1408, 49152, "DeepSeek-MoE-16B-style fine-grained experts")
    run(128, 2048, 768, 32768, "128 small experts")


if __name__ == "__main__":
    main()
