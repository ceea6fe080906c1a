"""Where do the GPT2-1.5B step's device copies / fills come from?  One step
under torch.profiler with Python stacks; prints the top call sites of
aten::copy_ / aten::fill_ / aten::add on CUDA (kernel-time weighted)."""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    dev = torch.device("cuda", 0)
    cfg = GPT2Config.named("gpt2-1.5b")
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model, lazy_zero_grad=True)
    opt = FusedAdamW(flat, lr=1e-4, max_grad_norm=1.0)
    data = torch.randint(0, cfg.vocab_size, (8, 1025), device=dev)

    def step():
        loss = model(data[:, :-1], data[:, 1:])
        loss.backward()
        opt.step()
        flat.zero_grad()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as p:
        step()
        torch.cuda.synchronize()
    agg = collections.Counter()
    cnt = collections.Counter()
    for e in p.events():
        if e.name not in ("aten::copy_", "aten::fill_", "aten::add_", "aten::add", "aten::contiguous", "aten::zero_",
                          "aten::_to_copy", "aten::clone"):
            continue
        stack = [s for s in (e.stack or []) if "dlrover_wuqiong_amd" in s or "bench" in s][:3]
        key = (e.name, str(e.input_shapes)[:80], " <- ".join(stack))
        agg[key] += e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
        cnt[key] += 1
    for k, v in agg.most_common(25):
        print(f"{v / 1000:8.2f} ms  x{cnt[k]:3d}  {k[0]}  {k[1]}  {k[2]}")
    # every CPU op that launched device work, by call count (per-layer ones x48)
    ops = collections.Counter()
    dt = collections.Counter()
    for e in p.events():
        t = e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total
        if e.name.startswith("aten::") and t > 0:
            ops[(e.name, str(e.input_shapes)[:90])] += 1
            dt[(e.name, str(e.input_shapes)[:90])] += t
    print("--- aten ops with device time, by count")
    for k, n in ops.most_common(40):
        print(f"x{n:4d}  {dt[k] / 1000:8.2f} ms  {k[0]}  {k[1]}")


if __name__ == "__main__":
    main()
