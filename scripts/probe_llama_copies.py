"""Which ops launch device copies in a Llama step (flat_zero2)?  torch.profiler
with Python stacks on a small Llama config (same per-layer structure as 8B)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dlrover_wuqiong_amd.atorch.auto_accelerate import auto_accelerate  # noqa: E402
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer  # noqa: E402

cfg = LlamaConfig.named("llama-tiny")
cfg.num_hidden_layers = 4
with torch.device("cuda"):
    m = Llama(cfg)
ok, res, _ = auto_accelerate(m, optim_func=torch.optim.AdamW, optim_args={"lr": 2e-5},
                             load_strategy=["module_replace", "half", ("flat_zero2", {"wrap_cls": (LlamaDecoderLayer,)})])
model, opt = res.model, res.optim
x = torch.randint(0, cfg.vocab_size, (1, 513), device="cuda")
for _ in range(3):
    loss = model(x[:, :-1], x[:, 1:])
    loss.backward()
    opt.step()
    opt.zero_grad()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    loss = model(x[:, :-1], x[:, 1:])
    loss.backward()
    opt.step()
    opt.zero_grad()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="count", row_limit=40, max_name_column_width=60))
print(prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=25, max_name_column_width=50,
                                                   max_src_column_width=160))
