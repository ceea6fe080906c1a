"""Llama-2 pre-training with FSDP through ``auto_accelerate`` (reference:
atorch/examples/llama2/fsdp_llama2.py): FSDP2 over the decoder layers,
bf16 autocast or pure-bf16 ("half"), activation checkpointing, optional FP8
GEMMs, fused HIP norms / flash attention / multi-tensor AdamW.

    dlrover-run --nproc_per_node=8 examples/llama2/fsdp_llama2.py --model llama2-7b \
        --per_device_train_batch_size 4 --block_size 4096 --precision bf16_amp --gradient_checkpointing
"""

import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402
from example_utils import llama_train_flops, print_rank_0, sync_and_time, synthetic_batches  # noqa: E402

import atorch  # noqa: E402
from atorch.auto import auto_accelerate  # noqa: E402
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Llama-2 FSDP pre-training (synthetic data)")
    p.add_argument("--model", default="llama-tiny", help="LlamaConfig.named() entry, e.g. llama2-7b")
    p.add_argument("--num_layers", type=int, default=0, help="override the layer count (0: the config's)")
    p.add_argument("--per_device_train_batch_size", type=int, default=2)
    p.add_argument("--block_size", type=int, default=128)
    p.add_argument("--max_steps", type=int, default=10)
    p.add_argument("--learning_rate", type=float, default=1e-4)
    p.add_argument("--precision", choices=["bf16_amp", "bf16", "fp32"], default="bf16_amp")
    p.add_argument("--gradient_checkpointing", action="store_true")
    p.add_argument("--fp8", action="store_true")
    p.add_argument("--no_fsdp", action="store_true")
    return p.parse_args(argv)


def optim_param_func(model):
    no_decay = ("norm.weight", "bias")
    return [{"params": [p for n, p in model.named_parameters() if not any(k in n for k in no_decay)],
             "weight_decay": 0.1},
            {"params": [p for n, p in model.named_parameters() if any(k in n for k in no_decay)],
             "weight_decay": 0.0}]


def main(argv=None):
    args = parse_args(argv)
    if int(os.getenv("WORLD_SIZE", "1")) > 1:
        atorch.init_distributed("nccl" if torch.cuda.is_available() else "gloo",
                                set_cuda_device_using_local_rank=True)
    cfg = LlamaConfig.named(args.model)
    if args.num_layers:
        cfg.num_hidden_layers = args.num_layers
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, args.block_size)
    torch.manual_seed(0)
    model = Llama(cfg)

    strategy = ["parallel_mode", "module_replace"]
    if not args.no_fsdp and atorch.world_size() > 1:
        strategy.append(("fsdp", {"atorch_wrap_cls": (LlamaDecoderLayer,), "sync_module_states": True,
                                  "use_orig_params": True, "limit_all_gathers": True, "forward_prefetch": True}))
    if args.precision == "bf16_amp":
        strategy.append(("amp_native", {"dtype": torch.bfloat16}))
    elif args.precision == "bf16":
        strategy.append(("half", "bf16"))
    if args.gradient_checkpointing:
        strategy.append(("checkpoint", {"wrap_class": (LlamaDecoderLayer,), "no_reentrant": True}))
    if args.fp8:
        strategy.append(("fp8", {"include": ("layers",)}))
    status, result, best = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": args.learning_rate},
                                           optim_param_func=optim_param_func, load_strategy=strategy,
                                           ignore_dryrun_on_load_strategy=True)
    assert status, "auto_accelerate failed"
    print_rank_0(f"strategy: {best.names()}")
    model, optim = result.model, result.optim
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    data = synthetic_batches(cfg.vocab_size, args.per_device_train_batch_size, args.block_size,
                             seed=atorch.rank() or 0)
    flops = llama_train_flops(args.per_device_train_batch_size, args.block_size, cfg.hidden_size, cfg.vocab_size,
                              cfg.intermediate_size, cfg.num_hidden_layers, args.gradient_checkpointing)
    losses, t = [], sync_and_time()
    for step in range(args.max_steps):
        batch = result.prepare_input(next(data), dev)
        optim.zero_grad()
        loss = model(batch["input_ids"], batch["labels"])
        loss.backward()
        optim.step()
        losses.append(float(loss.detach()))
        t2 = sync_and_time()
        print_rank_0(f"iter {step}: loss {losses[-1]:.4f}  {t2 - t:.3f}s  "
                     f"{flops / (t2 - t) / 1e12:.1f} TFLOP/s per device")
        t = t2
    return losses


if __name__ == "__main__":
    main()
