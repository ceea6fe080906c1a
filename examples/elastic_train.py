"""Elastic training example: flash checkpoint every step, restore from host
memory after a failure (used by the agent end-to-end tests and the goodput
experiment).

    dwamd-run --nnodes=1 --nproc-per-node=2 examples/elastic_train.py --steps 50

Runs on GPUs (RCCL) when available, else CPU/gloo.  With
``DWAMD_FAULT_INJECT_STEP``/``DWAMD_FAULT_INJECT_RANK`` set, that rank exits
at that step of the first run; the agent restarts the worker group and the
new processes resume from the in-memory checkpoint.
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
from dlrover_wuqiong_amd.trainer.elastic import maybe_inject_fault  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--ckpt-dir", default="/tmp/dwamd_elastic_example")
    p.add_argument("--out", default="")
    p.add_argument("--hidden", type=int, default=256)
    p.add_argument("--disk-every", type=int, default=0)
    p.add_argument("--step-sleep", type=float, default=0.0, help="slow steps down (fault-injection tests)")
    p.add_argument("--progress", default="", help="rank 0 writes the last finished step here")
    a = p.parse_args()
    t_start = time.time()
    cuda = torch.cuda.is_available()
    lr = int(os.getenv("LOCAL_RANK", "0"))
    dev = torch.device("cuda", lr) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    dist.init_process_group("nccl" if cuda else "gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(a.hidden, a.hidden), torch.nn.GELU(),
                                torch.nn.Linear(a.hidden, 1)).to(dev)
    ddp = torch.nn.parallel.DistributedDataParallel(model)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    ckpt = DdpCheckpointer(a.ckpt_dir)
    t_load = time.time()
    state = ckpt.load_checkpoint()
    t_load = time.time() - t_load
    start = 0
    if state:
        model.load_state_dict(state["model"])
        opt.load_state_dict(state["optimizer"])
        start = int(state["step"])
    g = torch.Generator().manual_seed(1234 + rank)
    x = torch.randn(64, a.hidden, generator=g).to(dev)
    y = x.sum(-1, keepdim=True) * 0.01
    loss = torch.zeros(())
    for step in range(start, a.steps):
        maybe_inject_fault(step)
        loss = torch.nn.functional.mse_loss(ddp(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        sd = {"model": model.state_dict(), "optimizer": opt.state_dict(), "step": step + 1}
        st = StorageType.DISK if a.disk_every and (step + 1) % a.disk_every == 0 else StorageType.MEMORY
        ckpt.save_checkpoint(step + 1, sd, storage_type=st)
        if a.progress and rank == 0:
            with open(a.progress, "w") as f:
                f.write(str(step + 1))
        if a.step_sleep:
            time.sleep(a.step_sleep)
    ckpt.wait_latest_checkpoint()
    dist.barrier()
    if a.out and rank == 0:
        with open(a.out, "a") as f:
            f.write(json.dumps({"restart": int(os.getenv("TORCHELASTIC_RESTART_COUNT", "0")), "start_step": start,
                                "final_loss": float(loss), "world": world, "load_sec": t_load,
                                "wall": time.time() - t_start}) + "\n")
    ckpt.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
