"""Which FP8 GEMM paths work on this torch / ROCm / gfx950: torch._scaled_mm
with OCP e4m3fn / e5m2 (and the fnuz types), layouts, bias, timing."""
import time

import torch

dev = "cuda"
print(torch.__version__, torch.version.hip, torch.cuda.get_device_name(0), flush=True)
M, N, K = 8192, 6400, 1600
a = torch.randn(M, K, device=dev)
b = torch.randn(N, K, device=dev)
ref = (a @ b.t())
for (ta, tb) in [(torch.float8_e4m3fn, torch.float8_e4m3fn), (torch.float8_e5m2, torch.float8_e4m3fn),
                 (torch.float8_e4m3fnuz, torch.float8_e4m3fnuz)]:
    try:
        a8 = a.to(ta)
        b8 = b.to(tb)
        one = torch.ones((), device=dev)
        y = torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        err = ((y.float() - ref).norm() / ref.norm()).item()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            y = torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 20
        print(ta, tb, "ok rel_err", round(err, 4), "us", round(dt * 1e6, 1), "TF/s", round(2 * M * N * K / dt / 1e12, 1),
              flush=True)
        try:
            bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
            y = torch._scaled_mm(a8, b8.t(), scale_a=one, scale_b=one, bias=bias, out_dtype=torch.bfloat16)
            print("  bias ok", flush=True)
        except Exception as e:
            print("  bias fail", repr(e)[:200], flush=True)
    except Exception as e:
        print(ta, tb, "FAIL", repr(e)[:300], flush=True)
ab = a.bfloat16()
bb = b.bfloat16()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    y = ab @ bb.t()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 20
print("bf16 us", round(dt * 1e6, 1), "TF/s", round(2 * M * N * K / dt / 1e12, 1), flush=True)
