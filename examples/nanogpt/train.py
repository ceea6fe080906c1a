"""nanoGPT elastic training with flash checkpoints (reference:
examples/pytorch/nanogpt/train.py): ElasticTrainer (fixed global batch
across scale events), ElasticDistributedSampler (resumes mid-epoch),
DdpCheckpointer saves to node shm every ``--save_memory_interval`` steps and
persists every ``--save_storage_interval`` steps; optional LoRA.

    dlrover-run --nnodes=1 --nproc_per_node=8 examples/nanogpt/train.py \
        --n_layer 12 --n_head 12 --n_embd 768 --block_size 1024 --batch_size 16

Data: ``--data_dir`` with a ``train.bin`` of uint16 tokens (nanoGPT's
prepare.py format) or, without one, random tokens.
"""

import argparse
import contextlib
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
from torch.nn.parallel import DistributedDataParallel as DDP  # noqa: E402
from torch.utils.data import DataLoader, Dataset  # noqa: E402

from dlrover.trainer.torch.elastic.sampler import ElasticDistributedSampler  # noqa: E402
from dlrover.trainer.torch.elastic.trainer import ElasticTrainer  # noqa: E402
from dlrover.trainer.torch.flash_checkpoint.ddp import DdpCheckpointer, StorageType  # noqa: E402
from dlrover_wuqiong_amd.atorch.lora import apply_lora, create_lora_config  # noqa: E402
from dlrover_wuqiong_amd.models.gpt2 import GPT2, GPT2Config  # noqa: E402


class TokenDataset(Dataset):
    def __init__(self, data: np.ndarray, block_size: int):
        self.data, self.block_size = data, block_size

    def __len__(self):
        return (len(self.data) - 1) // self.block_size

    def __getitem__(self, i):
        s = i * self.block_size
        chunk = torch.from_numpy(self.data[s: s + self.block_size + 1].astype(np.int64))
        return chunk[:-1], chunk[1:]


def load_tokens(data_dir: str, vocab: int, n_tokens: int) -> np.ndarray:
    path = os.path.join(data_dir or "", "train.bin")
    if data_dir and os.path.exists(path):
        return np.memmap(path, dtype=np.uint16, mode="r")
    return np.random.default_rng(0).integers(0, vocab, n_tokens, dtype=np.uint16)


def get_lr(it, a):
    if it < a.warmup_iters:
        return a.learning_rate * (it + 1) / max(1, a.warmup_iters)
    if it > a.lr_decay_iters:
        return a.min_lr
    r = (it - a.warmup_iters) / max(1, a.lr_decay_iters - a.warmup_iters)
    return a.min_lr + 0.5 * (1.0 + math.cos(math.pi * r)) * (a.learning_rate - a.min_lr)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--data_dir", default="")
    p.add_argument("--vocab_size", type=int, default=1024)
    p.add_argument("--synthetic_tokens", type=int, default=1 << 18)
    p.add_argument("--batch_size", type=int, default=8, help="micro-batch per rank")
    p.add_argument("--block_size", type=int, default=128)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--n_layer", type=int, default=2)
    p.add_argument("--n_head", type=int, default=4)
    p.add_argument("--n_embd", type=int, default=256)
    p.add_argument("--gradient_accumulation_steps", type=int, default=0, help="global; split over ranks")
    p.add_argument("--learning_rate", type=float, default=6e-4)
    p.add_argument("--max_iters", type=int, default=20)
    p.add_argument("--weight_decay", type=float, default=0.1)
    p.add_argument("--beta1", type=float, default=0.9)
    p.add_argument("--beta2", type=float, default=0.95)
    p.add_argument("--grad_clip", type=float, default=1.0)
    p.add_argument("--decay_lr", action="store_true")
    p.add_argument("--warmup_iters", type=int, default=0)
    p.add_argument("--lr_decay_iters", type=int, default=2000)
    p.add_argument("--min_lr", type=float, default=6e-5)
    p.add_argument("--lora_rank", type=int, default=None)
    p.add_argument("--lora_dropout", type=float, default=None)
    p.add_argument("--lora_alpha", type=float, default=None)
    p.add_argument("--lora_targets", type=str, default=None, help="comma-separated name fragments, e.g. c_attn")
    p.add_argument("--save_dir", default="/tmp/nanogpt_ckpt")
    p.add_argument("--save_memory_interval", type=int, default=5)
    p.add_argument("--save_storage_interval", type=int, default=20)
    p.add_argument("--log_interval", type=int, default=1)
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    world = int(os.getenv("WORLD_SIZE", "1"))
    local_rank = int(os.getenv("LOCAL_RANK", "0"))
    cuda = torch.cuda.is_available()
    device = torch.device("cuda", local_rank) if cuda else torch.device("cpu")
    if cuda:
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group("nccl" if cuda else "gloo")
    rank = dist.get_rank() if dist.is_initialized() else 0
    ctx = torch.autocast("cuda", dtype=torch.bfloat16) if cuda else contextlib.nullcontext()
    ga = max(1, a.gradient_accumulation_steps // world) if a.gradient_accumulation_steps else 1

    data = load_tokens(a.data_dir, a.vocab_size, a.synthetic_tokens)
    ds = TokenDataset(data, a.block_size)
    sampler = ElasticDistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True, seed=0)
    loader = DataLoader(ds, batch_size=a.batch_size, sampler=sampler, drop_last=True, pin_memory=cuda)

    torch.manual_seed(0)
    cfg = GPT2Config(vocab_size=a.vocab_size, n_positions=a.block_size, n_layer=a.n_layer, n_head=a.n_head,
                     n_embd=a.n_embd)
    model = GPT2(cfg).to(device)
    lora = create_lora_config(a)
    if lora is not None:
        wrapped = apply_lora(model, **lora)
        if rank == 0:
            print(f"LoRA {lora}: {len(wrapped)} linears adapted", flush=True)
    if world > 1:
        model = DDP(model, device_ids=[local_rank] if cuda else None)
    elastic = ElasticTrainer(model, dataloader=loader)
    optim = torch.optim.AdamW([p for p in model.parameters() if p.requires_grad], lr=a.learning_rate,
                              weight_decay=a.weight_decay, betas=(a.beta1, a.beta2))
    optim = elastic.prepare(optim)
    ckpt = DdpCheckpointer(a.save_dir)

    # resume: shm if this node holds a newer step, else storage
    step = 0
    t0 = time.time()
    state = ckpt.load_checkpoint()
    if state and "model" in state:
        (model.module if hasattr(model, "module") else model).load_state_dict(state["model"])
        try:
            optim.load_state_dict(state["optimizer"])
        except (ValueError, KeyError):  # e.g. LoRA fine-tuning from a base checkpoint
            if rank == 0:
                print("optimizer state not restored: different trainable parameters", flush=True)
        if "sampler" in state:
            sampler.load_state_dict(state["sampler"])
        step = int(state.get("step", 0))
        if rank == 0:
            print(f"resumed at step {step} in {time.time() - t0:.3f}s", flush=True)

    def state_dict():
        m = model.module if hasattr(model, "module") else model
        return {"model": m.state_dict(), "optimizer": optim.state_dict(), "step": step,
                "sampler": sampler.state_dict(step * ga, a.batch_size)}

    losses = []
    for epoch in range(a.epochs):
        sampler.set_epoch(epoch)
        for idx, (x, y) in enumerate(loader):
            x, y = x.to(device, non_blocking=True), y.to(device, non_blocking=True)
            lr = get_lr(step, a) if a.decay_lr else a.learning_rate
            for g in optim.param_groups:
                g["lr"] = lr
            t = time.time()
            with elastic.step():
                with ctx:
                    loss = model(x, y) / ga
                loss.backward()
                if (idx + 1) % ga == 0:
                    if a.grad_clip:
                        torch.nn.utils.clip_grad_norm_([p for p in model.parameters() if p.requires_grad],
                                                       a.grad_clip)
                    optim.step()
                    optim.zero_grad(set_to_none=True)
                    step += 1
            if (idx + 1) % ga:
                continue
            losses.append(float(loss.detach()) * ga)
            if rank == 0 and step % a.log_interval == 0:
                print(f"iter {step}: loss {losses[-1]:.4f}, time {(time.time() - t) * 1000:.1f}ms, lr {lr:.2e}",
                      flush=True)
            if step % a.save_memory_interval == 0:
                ts = time.time()
                ckpt.save_checkpoint(step, state_dict(), storage_type=StorageType.MEMORY)
                if rank == 0:
                    print(f"flash save (memory) step {step}: {time.time() - ts:.4f}s", flush=True)
            if step % a.save_storage_interval == 0:
                ckpt.save_checkpoint(step, state_dict(), storage_type=StorageType.DISK)
            if step >= a.max_iters:
                ckpt.close() if hasattr(ckpt, "close") else None
                return losses
    return losses


if __name__ == "__main__":
    main()
