"""Mixture-of-Experts training: sparse upcycling of a dense Llama, expert
parallelism inside a node, MoE-aware data parallelism across EP groups
(reference: atorch/modules/moe -- inject.replace_with_moe, MOELayer,
MoEMixtureDistributedDataParallel).

    dlrover-run --nproc_per_node=8 examples/moe/train_moe.py --ep 8 --experts 16
    python -m torch.distributed.run --nproc-per-node 4 examples/moe/train_moe.py --ep 2   # EP 2 x DP 2

The dense model is built (or loaded), every SwiGLU FFN becomes an MoE layer
whose experts start as copies of it (the MoE model computes the dense
function at step 0), then trains with the router's load-balance loss.
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import atorch  # noqa: E402
from atorch.auto import auto_accelerate  # noqa: E402
from atorch.modules.moe.inject import replace_with_moe  # noqa: E402
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaMLP  # noqa: E402
from dlrover_wuqiong_amd.parallel.moe import moe_aux_loss  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama-tiny")
    p.add_argument("--experts", type=int, default=4)
    p.add_argument("--top_k", type=int, default=2)
    p.add_argument("--ep", type=int, default=1, help="expert-parallel degree (consecutive ranks)")
    p.add_argument("--capacity_factor", type=float, default=0.0, help="0: dropless")
    p.add_argument("--noise_std", type=float, default=1e-3, help="upcycling noise on the expert copies")
    p.add_argument("--batch", type=int, default=2, help="per rank")
    p.add_argument("--seq", type=int, default=64)
    p.add_argument("--steps", type=int, default=6)
    p.add_argument("--lr", type=float, default=1e-3)
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    world = int(os.getenv("WORLD_SIZE", "1"))
    if world > 1:
        atorch.init_distributed("nccl" if torch.cuda.is_available() else "gloo",
                                set_cuda_device_using_local_rank=True)
    rank = dist.get_rank() if dist.is_initialized() else 0
    ep_group = None
    if a.ep > 1:
        assert world % a.ep == 0, "world size must be a multiple of --ep"
        for i in range(world // a.ep):  # every rank creates every EP group
            g = dist.new_group(list(range(i * a.ep, (i + 1) * a.ep)))
            if rank // a.ep == i:
                ep_group = g
    cfg = LlamaConfig.named(a.model)
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, a.seq)
    torch.manual_seed(0)  # the same dense weights on every rank
    model = Llama(cfg)
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    ids = torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), generator=torch.Generator().manual_seed(rank))
    with torch.no_grad():
        dense_loss = float(model(ids[:, :-1], ids[:, 1:]))
    names = replace_with_moe(model, LlamaMLP, a.experts, a.top_k, ep_group=ep_group,
                             capacity_factor=a.capacity_factor, noise_std=a.noise_std)
    with torch.no_grad():
        moe_loss = float(model(ids[:, :-1], ids[:, 1:]))
    if rank == 0:
        print(f"upcycled {len(names)} FFNs into {a.experts} experts (EP {a.ep}); "
              f"loss dense {dense_loss:.4f} -> MoE {moe_loss:.4f} at step 0", flush=True)
    strategy = ["parallel_mode", "ddp"] if world > 1 else []
    if torch.cuda.is_available():
        strategy = ["module_replace", ("amp_native", {"dtype": torch.bfloat16})] + strategy
    ok, res, best = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": a.lr}, load_strategy=strategy,
                                    ignore_dryrun_on_load_strategy=True)
    assert ok
    m, opt = res.model, res.optim
    losses = []
    for step in range(a.steps):
        b = ids.to(dev)
        loss = m(b[:, :-1], b[:, 1:])
        (loss + moe_aux_loss(model)).backward()
        opt.step()
        opt.zero_grad()
        losses.append(float(loss))
        if rank == 0:
            print(f"step {step}: loss {losses[-1]:.4f} aux {float(moe_aux_loss(model)):.4f}", flush=True)
    if rank == 0:
        print(f"first_loss={losses[0]:.4f} last_loss={losses[-1]:.4f} strategy={best.names()}", flush=True)
    return dense_loss, moe_loss, losses


if __name__ == "__main__":
    main()
