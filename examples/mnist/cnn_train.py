"""MNIST-shaped CNN under elastic data parallelism (reference:
examples/pytorch/mnist/cnn_train.py): ElasticDataLoader whose batch size
follows the agent's parallel-config tuner, ElasticTrainer keeping the global
batch fixed when ranks come and go, resumable sampler, flash checkpoints.

    dlrover-run --nnodes=1:4 --nproc_per_node=2 --max-restarts 3 examples/mnist/cnn_train.py

Data: 28x28 digit-like images generated from 10 random stroke templates
(no download).
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from torch.utils.data import TensorDataset  # noqa: E402

from dlrover.trainer.torch.elastic.dataloader import ElasticDataLoader  # noqa: E402
from dlrover.trainer.torch.elastic.sampler import ElasticDistributedSampler  # noqa: E402
from dlrover.trainer.torch.elastic.trainer import ElasticTrainer  # noqa: E402
from dlrover.trainer.torch.flash_checkpoint.ddp import DdpCheckpointer, StorageType  # noqa: E402


class Net(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv1 = nn.Conv2d(1, 32, 3, 1)
        self.conv2 = nn.Conv2d(32, 64, 3, 1)
        self.fc1 = nn.Linear(9216, 128)
        self.fc2 = nn.Linear(128, 10)

    def forward(self, x):
        x = F.relu(self.conv1(x))
        x = F.max_pool2d(F.relu(self.conv2(x)), 2)
        x = F.relu(self.fc1(torch.flatten(x, 1)))
        return self.fc2(x)


def digits(n, seed=0):
    g = torch.Generator().manual_seed(seed)
    templates = (torch.rand(10, 1, 28, 28, generator=g) > 0.8).float()
    y = torch.randint(0, 10, (n,), generator=g)
    x = templates[y] + 0.3 * torch.randn(n, 1, 28, 28, generator=g)
    return TensorDataset(x, y)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--batch_size", type=int, default=32)
    p.add_argument("--num_epochs", type=int, default=1)
    p.add_argument("--samples", type=int, default=2048)
    p.add_argument("--learning_rate", type=float, default=0.05)
    p.add_argument("--max_steps", type=int, default=0)
    p.add_argument("--save_memory_interval", type=int, default=10)
    p.add_argument("--save_storage_interval", type=int, default=50)
    p.add_argument("--checkpoint_dir", default="/tmp/mnist_ckpt")
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    world, rank = int(os.getenv("WORLD_SIZE", "1")), int(os.getenv("RANK", "0"))
    cuda = torch.cuda.is_available()
    dev = torch.device("cuda", int(os.getenv("LOCAL_RANK", "0"))) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl" if cuda else "gloo")
    ds = digits(a.samples)
    sampler = ElasticDistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True)
    loader = ElasticDataLoader(ds, batch_size=a.batch_size, sampler=sampler, drop_last=True)
    torch.manual_seed(0)
    model = Net().to(dev)
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[dev.index] if cuda else None)
    elastic = ElasticTrainer(model, dataloader=loader)
    opt = elastic.prepare(torch.optim.SGD(model.parameters(), lr=a.learning_rate, momentum=0.9))
    ckpt = DdpCheckpointer(a.checkpoint_dir)
    step = 0
    st = ckpt.load_checkpoint()
    if st and "model" in st:
        (model.module if hasattr(model, "module") else model).load_state_dict(st["model"])
        opt.load_state_dict(st["optimizer"])
        sampler.load_state_dict(st["sampler"])
        step = st["step"]
        if rank == 0:
            print(f"resumed at step {step}", flush=True)
    losses = []
    for epoch in range(a.num_epochs):
        sampler.set_epoch(epoch)
        loader.load_config()  # batch size from the agent's tuner, if it changed
        for x, y in loader:
            x, y = x.to(dev), y.to(dev)
            with elastic.step():
                loss = F.cross_entropy(model(x), y)
                loss.backward()
                opt.step()
                opt.zero_grad()
            step += 1
            losses.append(float(loss))
            if rank == 0 and step % 10 == 0:
                print(f"step {step}: loss {losses[-1]:.4f}", flush=True)
            if step % a.save_memory_interval == 0 or step % a.save_storage_interval == 0:
                sd = {"model": (model.module if hasattr(model, "module") else model).state_dict(),
                      "optimizer": opt.state_dict(), "step": step,
                      "sampler": sampler.state_dict(step, loader.batch_sampler.batch_size)}
                kind = StorageType.DISK if step % a.save_storage_interval == 0 else StorageType.MEMORY
                ckpt.save_checkpoint(step, sd, storage_type=kind)
            if a.max_steps and step >= a.max_steps:
                break
        if a.max_steps and step >= a.max_steps:
            break
    if rank == 0:
        print(f"first_loss={losses[0]:.4f} last_loss={sum(losses[-5:]) / len(losses[-5:]):.4f}", flush=True)
    return losses


if __name__ == "__main__":
    main()
