"""One GPT2 FC1-shaped Fp8Linear fwd+bwd loop for a rocprofv3 kernel trace."""
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.ops import fp8  # noqa: E402

T, K, N = 8192, 1600, 6400
lin = nn.Linear(K, N, device="cuda", dtype=torch.bfloat16)
f8 = fp8.Fp8Linear(lin)
x = torch.randn(T, K, device="cuda", dtype=torch.bfloat16, requires_grad=True)
g = torch.randn(T, N, device="cuda", dtype=torch.bfloat16)
for _ in range(10):
    f8(x).backward(g)
    fp8.fp8_update()
torch.cuda.synchronize()
print("done")
