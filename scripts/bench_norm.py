"""Norm backward micro-benchmark (GPT2-1.5B / Llama shapes): one-pass fused
kernel vs row pass + column-reduction pass (DWAMD_NORM_BWD_2PASS=1); for
H < 2048 the block-partials path vs the atomic-combined one
(DWAMD_NORM_BWD_PART_OFF=1)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from dlrover_wuqiong_amd.ops.norm import layer_norm, rms_norm  # noqa: E402


def main():
    for R, H, rms in [(8192, 1600, False), (16384, 1600, False), (8192, 1024, True), (16384, 4096, True)]:
        x = torch.randn(R, H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        w = torch.ones(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        b = torch.zeros(H, device="cuda", dtype=torch.bfloat16, requires_grad=True)
        y = rms_norm(x, w, 1e-6) if rms else layer_norm(x, w, b, 1e-5)
        dy = torch.randn_like(y)
        for _ in range(3):
            torch.autograd.grad(y, [x, w], dy, retain_graph=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            torch.autograd.grad(y, [x, w], dy, retain_graph=True)
        e1.record()
        torch.cuda.synchronize()
        us = 1000 * e0.elapsed_time(e1) / n
        gbs = 3 * R * H * 2 / (us * 1e-6) / 1e9  # x, dy read + dx written
        print(json.dumps({"R": R, "H": H, "rms": rms, "bwd_us": round(us, 1), "hbm_gbs": round(gbs),
                          "two_pass": os.environ.get("DWAMD_NORM_BWD_2PASS", "0"),
                          "part_off": os.environ.get("DWAMD_NORM_BWD_PART_OFF", "0")}), flush=True)


if __name__ == "__main__":
    main()
