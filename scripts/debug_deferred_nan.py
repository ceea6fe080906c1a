"""Debug: NaNs after the deferred-restore first step (tests/test_flash_ckpt_gpu.py
test_gpu_deferred_optimizer_restore_orders_the_first_step).  Prints where the
first NaN appears: after the first plain step, after the restore, after the
step behind the deferred restore."""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def nan(t):
    return int(torch.isnan(t.float()).sum())


def main():
    from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType
    from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer
    from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config
    from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW
    from dlrover_wuqiong_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    cfg = GPT2Config.named("gpt2-tiny")
    with torch.device("cuda"):
        model = GPT2(cfg)
    model.to(torch.bfloat16)
    flat = FlatParams(model)
    opt = FusedAdamW(flat, lr=1e-3)
    x = torch.randint(0, cfg.vocab_size, (2, 65), device="cuda", generator=torch.Generator("cuda").manual_seed(7))

    def step(tag):
        loss = model(x[:, :-1], x[:, 1:])
        loss.backward()
        g = nan(flat.grad)
        opt.step()
        flat.zero_grad()
        torch.cuda.synchronize()
        print(tag, "loss", float(loss), "nan grad", g, "nan data", nan(flat.data), "nan m", nan(opt.exp_avg),
              "nan v", nan(opt.exp_avg_sq), "nan master", nan(opt.master), flush=True)

    for i in range(3):
        step(f"plain{i}")
    d = tempfile.mkdtemp()
    ck = DdpCheckpointer(os.path.join(d, "ck"))
    state = lambda: {"model": model.state_dict(), "optimizer": opt.state_dict()}  # noqa
    assert ck.save_checkpoint(5, state(), storage_type=StorageType.MEMORY)
    ck.wait_latest_checkpoint()
    ck.load_checkpoint(target=state())
    torch.cuda.synchronize()
    print("after load: nan data", nan(flat.data), "m", nan(opt.exp_avg), "v", nan(opt.exp_avg_sq),
          "master", nan(opt.master), flush=True)
    step("after_load")
    flat.data.zero_()
    opt.exp_avg.fill_(3.0)
    opt.master.fill_(-1.0)
    ck.load_checkpoint(target=state())
    print("deferred:", ck.engine.last_deferred_restore is not None, flush=True)
    step("behind_deferred")
    ck.close()


if __name__ == "__main__":
    main()
