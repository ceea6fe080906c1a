"""GPT-2 elastic training with flash checkpoints (launch with dwamd-run).

    dwamd-run --nnodes=1 --nproc-per-node=8 examples/train_gpt2_elastic.py \
        --model gpt2-1.5b --steps 200 --ckpt-interval 4

Each rank logs one JSON line per finished step (``--step-log``), which the
goodput experiment (scripts/goodput_experiment.py) turns into
useful-time / wall-time under an injected failure.  After a restart the
workers restore model + optimizer in place from the node's shared memory
(sliced H2D + xGMI all-gather), falling back to storage.
"""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dlrover_wuqiong_amd.flash_checkpoint.checkpointer import StorageType  # noqa: E402
from dlrover_wuqiong_amd.flash_checkpoint.ddp import DdpCheckpointer  # noqa: E402
from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config  # noqa: E402
from dlrover_wuqiong_amd.optimizers.fused import FusedAdamW  # noqa: E402
from dlrover_wuqiong_amd.parallel.ddp import FlatDDP  # noqa: E402
from dlrover_wuqiong_amd.parallel.flat import FlatParams  # noqa: E402
from dlrover_wuqiong_amd.trainer.elastic import maybe_inject_fault  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gpt2-1.5b")
    p.add_argument("--micro-batch", type=int, default=8)
    p.add_argument("--seq", type=int, default=1024)
    p.add_argument("--steps", type=int, default=60)
    p.add_argument("--ckpt-interval", type=int, default=4)
    p.add_argument("--disk-interval", type=int, default=0)
    p.add_argument("--ckpt-dir", default="/tmp/dwamd_gpt2_ckpt")
    p.add_argument("--step-log", default="")
    a = p.parse_args()
    t_proc = time.time()
    lr = int(os.getenv("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", lr) if cuda else torch.device("cpu")
    tl = {}
    if cuda:
        torch.cuda.set_device(dev)
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    tl["cuda_init"] = time.time() - t_proc
    world = int(os.getenv("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("nccl" if cuda else "gloo", device_id=dev if cuda else None)
    tl["pg_init"] = time.time() - t_proc
    rank = int(os.getenv("RANK", "0"))
    dtype = torch.bfloat16 if cuda else torch.float32
    cfg = GPT2Config.named(a.model)
    cfg.n_positions = max(cfg.n_positions, a.seq)
    torch.manual_seed(1234)
    with torch.device(dev):
        model = GPT2(cfg)
    model.to(dtype)
    flat = FlatParams(model, dtype=dtype, device=dev, lazy_zero_grad=True)
    opt = FusedAdamW(flat, lr=1e-4, betas=(0.9, 0.95), weight_decay=0.1, max_grad_norm=1.0)
    ddp = FlatDDP(model, flat)
    opt.grad_scale = 1.0 / world
    tl["model_opt"] = time.time() - t_proc
    ckpt = DdpCheckpointer(a.ckpt_dir)
    tl["ckpt_init"] = time.time() - t_proc

    def state(step_t):
        return {"model": model.state_dict(), "optimizer": opt.state_dict(), "step": step_t}

    t_restore = time.time()
    restored = ckpt.load_checkpoint(target=state(0))
    if cuda:
        torch.cuda.synchronize()
    t_restore = time.time() - t_restore
    start = int(restored.get("step", 0)) if restored else 0
    g = torch.Generator().manual_seed(rank)
    data = torch.randint(0, cfg.vocab_size, (4, a.micro_batch, a.seq + 1), generator=g).to(dev)
    log = open(a.step_log, "a") if a.step_log and rank == 0 else None
    if log:
        log.write(json.dumps({"event": "start", "restart": int(os.getenv("TORCHELASTIC_RESTART_COUNT", "0")),
                              "start_step": start, "t": time.time(), "proc_start": t_proc,
                              "restore_sec": t_restore, "timeline": tl}) + "\n")
        log.flush()
    for step in range(start, a.steps):
        maybe_inject_fault(step)
        b = data[step % 4]
        loss = ddp(b[:, :-1], b[:, 1:])
        loss.backward()
        ddp.finish_gradient_sync()
        opt.step()
        flat.zero_grad()
        if cuda:
            torch.cuda.current_stream().synchronize()
        t_end = time.time()
        if (step + 1) % a.ckpt_interval == 0:
            st = (StorageType.DISK if a.disk_interval and (step + 1) % a.disk_interval == 0
                  else StorageType.MEMORY)
            ckpt.save_checkpoint(step + 1, state(step + 1), storage_type=st)
            if cuda:
                torch.cuda.current_stream().synchronize()
        if log:
            log.write(json.dumps({"event": "step", "step": step + 1, "t": time.time(), "t_train_end": t_end}) + "\n")
            log.flush()
    ckpt.wait_latest_checkpoint()
    if log:
        log.write(json.dumps({"event": "done", "t": time.time(), "loss": float(loss.detach())}) + "\n")
        log.close()
    ckpt.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
