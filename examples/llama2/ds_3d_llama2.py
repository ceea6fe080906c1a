"""Llama-2 with tensor x pipeline x data parallelism in one
``auto_accelerate`` strategy (reference: atorch/examples/llama2/
ds_3d_llama2.py, there on DeepSpeed's pipeline engine): Megatron TP layers
rebuilt from the unsharded model, 1F1B pipeline over decoder-layer stages,
gradient averaging over the data group; ``model.train_batch(data_iter)``.

    dlrover-run --nproc_per_node=8 examples/llama2/ds_3d_llama2.py --model llama2-7b \
        --model_parallel_size 2 --pipeline_parallel_size 2 --block_size 4096
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
from atorch.auto.opt_lib.ds_3d_parallel_optimization import DeepSpeed3DParallelConfig  # noqa: E402
from atorch.utils.manual_tp_utils import TPInfo  # noqa: E402
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig  # noqa: E402


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Llama-2 3D-parallel pre-training (synthetic data)")
    p.add_argument("--model", default="llama-tiny")
    p.add_argument("--num_layers", type=int, default=0)
    p.add_argument("--model_parallel_size", type=int, default=1)
    p.add_argument("--pipeline_parallel_size", type=int, default=1)
    p.add_argument("--micro_batch_size", type=int, default=1)
    p.add_argument("--gradient_accumulation_steps", type=int, default=2, help="micro-batches per pipeline step")
    p.add_argument("--block_size", type=int, default=64)
    p.add_argument("--max_steps", type=int, default=5)
    p.add_argument("--learning_rate", type=float, default=1e-4)
    return p.parse_args(argv)


def llama_tpinfo():
    info = TPInfo()
    info.shard_col("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj", "mlp.gate_proj", "mlp.up_proj")
    info.shard_row("self_attn.o_proj", "mlp.down_proj")
    info.shard_vocab("embed_tokens")
    info.shrink({"self_attn": {"num_heads", "num_key_value_heads", "hidden_size"}})
    return info


def main(argv=None):
    args = parse_args(argv)
    atorch.init_distributed("nccl" if torch.cuda.is_available() else "gloo", set_cuda_device_using_local_rank=True)
    t, p = args.model_parallel_size, args.pipeline_parallel_size
    d = atorch.world_size() // (t * p)
    print_rank_0(f"3D parallel: tensor {t}, pipeline {p}, data {d}")
    cfg = LlamaConfig.named(args.model)
    if args.num_layers:
        cfg.num_hidden_layers = args.num_layers
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, args.block_size)
    torch.manual_seed(0)
    model = Llama(cfg)
    ds_cfg = DeepSpeed3DParallelConfig(tpinfo=llama_tpinfo(),
                                       ds_config={"gradient_accumulation_steps": args.gradient_accumulation_steps,
                                                  "train_micro_batch_size_per_gpu": args.micro_batch_size},
                                       batch_fn=lambda b: (b["input_ids"], b["labels"]))
    strategy = [("parallel_mode", ([("tensor", t), ("pipeline", p), ("data", d)], None)),
                ("deepspeed_3d_parallel", ds_cfg)]
    status, result, best = auto_accelerate(model, torch.optim.AdamW, optim_args={"lr": args.learning_rate},
                                           load_strategy=strategy, ignore_dryrun_on_load_strategy=True)
    assert status, "auto_accelerate failed"
    model, optim = result.model, result.optim
    dev = "cuda" if torch.cuda.is_available() else "cpu"
    from dlrover_wuqiong_amd.atorch import distributed as adist

    data = (result.prepare_input(b, dev) for b in synthetic_batches(
        cfg.vocab_size, args.micro_batch_size, args.block_size, seed=adist.parallel_rank("data") or 0))
    gbs = args.micro_batch_size * args.gradient_accumulation_steps * d
    flops = llama_train_flops(gbs, args.block_size, cfg.hidden_size, cfg.vocab_size, cfg.intermediate_size,
                              cfg.num_hidden_layers)
    print_rank_0(f"global batch {gbs}")
    losses, ts = [], sync_and_time()
    last = model.stage == model.num_stages - 1 if hasattr(model, "stage") else True
    for it in range(args.max_steps):
        optim.zero_grad()
        loss = model.train_batch(data) if hasattr(model, "train_batch") else None
        optim.step()
        # the last stage holds the loss; share it for the log
        lt = torch.tensor([float(loss) if (loss is not None and last) else 0.0, 1.0 if last else 0.0])
        if torch.distributed.is_initialized():
            torch.distributed.all_reduce(lt)
        losses.append(float(lt[0] / max(1.0, float(lt[1]))))
        t2 = sync_and_time()
        print_rank_0(f"iter {it}: loss {losses[-1]:.4f}  {t2 - ts:.3f}s  "
                     f"{flops / (t2 - ts) / atorch.world_size() / 1e12:.2f} TFLOP/s per device")
        ts = t2
    return losses


if __name__ == "__main__":
    main()
