"""auto_accelerate example: toy / GPT-2 / Llama trained through ATorch's
``auto_accelerate`` API with a user-chosen strategy (reference:
atorch/examples/auto_accelerate/train.py -- same flags, same flow).

    # 1 process (GPU if present, else CPU)
    python examples/auto_accelerate/train.py --model_type llama --load_strategy --use_amp
    # 8 GPUs, FSDP + activation checkpointing + bf16 autocast
    dlrover-run --nproc_per_node=8 examples/auto_accelerate/train.py --model_type gpt2 \
        --distributed --load_strategy --use_fsdp --use_checkpointing --use_amp
    # HSDP with local SGD (zero x data mesh, >= 4 ranks)
    dlrover-run --nproc_per_node=8 examples/auto_accelerate/train.py --model_type llama \
        --distributed --load_strategy --use_fsdp --use_local_sgd --local_sgd_sync_interval 4

Everything is imported through the reference's package paths (``atorch.*``),
which this framework provides.
"""

import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import torch  # noqa: E402
from data import get_dataloader_args, get_dataset  # noqa: E402
from modeling import (ModelType, get_loss_func, get_model, get_model_input_format, get_model_type,  # noqa: E402
                      get_module_type)
from torch.utils.data import DataLoader  # noqa: E402
from torch.utils.data.distributed import DistributedSampler  # noqa: E402

import atorch  # noqa: E402
from atorch.auto.accelerate import auto_accelerate  # noqa: E402
from atorch.auto.model_context import get_data_partition_rank_and_size  # noqa: E402
from atorch.common.util_func import data_to_device  # noqa: E402


def optim_grouped_param_func(model):
    decay = [p for n, p in model.named_parameters() if "bias" not in n]
    no_decay = [p for n, p in model.named_parameters() if "bias" in n]
    return [{"params": decay, "weight_decay": 0.01}, {"params": no_decay, "weight_decay": 0.0}]


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="auto_accelerate example")
    p.add_argument("--model_type", type=str, required=True, help="toy | gpt2 | llama")
    p.add_argument("--datasize", type=int, default=200)
    p.add_argument("--epoch", type=int, default=2)
    p.add_argument("--max_steps", type=int, default=0, help="stop after this many steps (0: run every epoch)")
    p.add_argument("--hidden_size", type=int, default=256)
    p.add_argument("--head_num", type=int, default=4)
    p.add_argument("--layer_num", type=int, default=3)
    p.add_argument("--seq_length", type=int, default=64)
    p.add_argument("--batchsize", type=int, default=8, help="global batch")
    p.add_argument("--in_size", type=int, default=16)
    p.add_argument("--out_size", type=int, default=16)
    p.add_argument("--distributed", action="store_true")
    p.add_argument("--user_created_dataloader", action="store_true")
    p.add_argument("--load_strategy", action="store_true")
    p.add_argument("--optim_grouped_params", action="store_true")
    p.add_argument("--log_interval", type=int, default=10)
    p.add_argument("--use_fsdp", action="store_true")
    p.add_argument("--use_flat_fsdp", action="store_true",
                   help="flat-unit FSDP (one flat buffer per layer, in-place collectives, fused optimizer)")
    p.add_argument("--use_amp", action="store_true")
    p.add_argument("--use_fp8", action="store_true")
    p.add_argument("--use_checkpointing", action="store_true")
    p.add_argument("--use_module_replace", action="store_true")
    p.add_argument("--use_local_sgd", action="store_true")
    p.add_argument("--local_sgd_sync_interval", type=int, default=1)
    p.add_argument("--local_sgd_warmup_steps", type=int, default=0)
    p.add_argument("--outer_optim_class", choices=["none", "sgd"], default="none")
    return p.parse_args(argv)


def build_strategy(args, model_type):
    strategy = []
    world = int(os.getenv("WORLD_SIZE", "1"))
    if args.distributed:
        if args.use_local_sgd:
            if world < 4 or world % 2:
                raise RuntimeError("local SGD needs an even world size >= 4 (zero x data mesh)")
            strategy.append(("parallel_mode", ([("zero", world // 2), ("data", 2)], None)))
        else:
            strategy.append("parallel_mode")
    if args.use_module_replace:
        strategy.append("module_replace")
    if args.use_fsdp:
        fsdp_config = {"sync_module_states": True, "limit_all_gathers": True, "forward_prefetch": True,
                       "atorch_wrap_cls": (get_module_type(model_type),)}
        if args.optim_grouped_params:
            fsdp_config["use_orig_params"] = True
        if args.use_local_sgd:
            fsdp_config.update(use_local_sgd=True, local_sgd_sync_interval=args.local_sgd_sync_interval,
                               local_sgd_warmup_steps=args.local_sgd_warmup_steps,
                               outer_optim_class=torch.optim.SGD if args.outer_optim_class == "sgd" else None,
                               outer_optim_kwargs={"lr": 0.7, "momentum": 0.8, "nesterov": True})
        strategy.append(("fsdp", fsdp_config))
    if args.use_flat_fsdp:
        strategy.append(("flat_fsdp", {"wrap_cls": (get_module_type(model_type),), "reshard_after_forward": True}))
    if args.use_amp:
        strategy.append(("amp_native", {"dtype": torch.bfloat16}))
    if args.use_checkpointing:
        strategy.append(("checkpoint", {"wrap_class": (get_module_type(model_type),), "no_reentrant": True}))
    if args.use_fp8:
        if model_type == ModelType.TOY and (args.in_size % 16 or args.out_size % 16 or args.batchsize % 16):
            print("fp8 ignored: the toy model's in/out sizes and batch must be multiples of 16")
        else:
            strategy.append(("fp8", {"include": ("layers", "linears", "first_linear", "h.")}))
    return strategy


def train(args):
    model_type = get_model_type(args.model_type)
    if model_type is None:
        raise SystemExit(f"{args.model_type}: unsupported model type")
    if args.distributed:
        if torch.cuda.is_available():
            atorch.init_distributed("nccl", set_cuda_device_using_local_rank=True)
        else:
            atorch.init_distributed("gloo")
    device = "cuda" if torch.cuda.is_available() else "cpu"
    torch.manual_seed(0)
    if model_type == ModelType.TOY:
        model_config = {"in_features": args.in_size, "out_features": args.out_size, "num_linears": args.layer_num}
    else:
        model_config = {"hidden_size": args.hidden_size, "head_num": args.head_num, "layer_num": args.layer_num,
                        "seq_length": args.seq_length}
    model = get_model(model_type, model_config)
    loss_func = get_loss_func(model_type)
    dataset = get_dataset(model_type, seq_length=args.seq_length, input_size=args.in_size,
                          output_size=args.out_size, datasize=args.datasize)
    dataloader_args = get_dataloader_args(model_type, batch_size=args.batchsize)
    strategy = build_strategy(args, model_type) if args.load_strategy else None
    optim_func = atorch.optimizers.AGD if model_type == ModelType.LLAMA else torch.optim.AdamW
    model_input_format = get_model_input_format(model_type)

    status, res, best_strategy = auto_accelerate(
        model, optim_func=optim_func, dataset=None if args.user_created_dataloader else dataset,
        loss_func=loss_func, prepare_input=data_to_device, model_input_format=model_input_format,
        optim_args={"lr": 1e-3}, optim_param_func=optim_grouped_param_func if args.optim_grouped_params else None,
        dataloader_args=None if args.user_created_dataloader else dataloader_args, load_strategy=strategy,
        ignore_dryrun_on_load_strategy=args.load_strategy)
    assert status
    model, optim, dataloader = res.model, res.optim, res.dataloader
    loss_func, prepare_input = res.loss_func, res.prepare_input
    if args.user_created_dataloader:
        sampler = None
        rank, dp_size = get_data_partition_rank_and_size()
        if dp_size > 1:
            dataloader_args["batch_size"] //= dp_size  # global batch -> per replica
            sampler = DistributedSampler(dataset, shuffle=dataloader_args.pop("shuffle", False),
                                         num_replicas=dp_size, rank=rank)
        dataloader = DataLoader(dataset, sampler=sampler, **dataloader_args)

    is_main = (atorch.rank() or 0) == 0
    if is_main:
        print(f"strategy: {best_strategy.names()}")
    step, losses, t0 = 0, [], time.time()
    for _ in range(args.epoch):
        for batch in dataloader:
            optim.zero_grad()
            batch = prepare_input(batch, device)
            if model_input_format == "unpack_dict":
                outputs = model(**batch)
            elif model_input_format == "unpack_sequence":
                outputs = model(*batch)
            else:
                outputs = model(batch)
            loss = loss_func(batch, outputs)
            loss.backward()
            optim.step()
            losses.append(float(loss))
            step += 1
            if step % args.log_interval == 0 and is_main:
                dt = (time.time() - t0) / args.log_interval
                print(f"[step={step - 1}] loss {losses[-1]:.4f}  {dt:.4f} sec/step", flush=True)
                t0 = time.time()
            if args.max_steps and step >= args.max_steps:
                break
        if args.max_steps and step >= args.max_steps:
            break
    if is_main:
        print(f"Finished training! steps={step} first_loss={losses[0]:.4f} last_loss={losses[-1]:.4f}", flush=True)
    return losses


if __name__ == "__main__":
    train(parse_args())
