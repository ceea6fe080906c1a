"""Llama-2 causal-LM training with AtorchTrainer (reference:
atorch/examples/llama2_7b_ATorchTrainer/llama2_clm_atorch_trainer.py):
HF-style ``AtorchArguments`` -> auto_accelerate strategy (FSDP / DDP, bf16
autocast, activation checkpointing), flash checkpoints every
``--save_steps``, resume with ``--resume_from_checkpoint``, optional LoRA.

    dlrover-run --nproc_per_node=8 examples/llama2_trainer/llama2_clm_atorch_trainer.py \
        --model llama2-7b --atorch_opt fsdp --bf16 --gradient_checkpointing --max_steps 1000
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402
from torch.utils.data import Dataset  # noqa: E402

import atorch  # noqa: E402
from atorch.trainer import AtorchArguments, AtorchTrainer  # noqa: E402
from dlrover_wuqiong_amd.atorch.lora import apply_lora, lora_state_dict  # noqa: E402
from dlrover_wuqiong_amd.models.llama import Llama, LlamaConfig, LlamaDecoderLayer  # noqa: E402


class CLMDataset(Dataset):
    """Fixed-length token blocks (random tokens; swap in a tokenised corpus)."""

    def __init__(self, vocab, block, n, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.data = torch.randint(0, vocab, (n, block + 1), generator=g)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, i):
        return {"ids": self.data[i, :-1], "targets": self.data[i, 1:]}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="llama-tiny")
    p.add_argument("--num_layers", type=int, default=0)
    p.add_argument("--block_size", type=int, default=64)
    p.add_argument("--samples", type=int, default=256)
    p.add_argument("--output_dir", default="/tmp/llama2_atorch_trainer")
    p.add_argument("--per_device_train_batch_size", type=int, default=4)
    p.add_argument("--max_steps", type=int, default=10)
    p.add_argument("--learning_rate", type=float, default=3e-4)
    p.add_argument("--save_steps", type=int, default=5)
    p.add_argument("--logging_steps", type=int, default=1)
    p.add_argument("--atorch_opt", default="fsdp", choices=["fsdp", "ddp", "zero2", "zero1", "none"])
    p.add_argument("--bf16", action="store_true")
    p.add_argument("--gradient_checkpointing", action="store_true")
    p.add_argument("--resume_from_checkpoint", action="store_true")
    p.add_argument("--lora_rank", type=int, default=0)
    return p.parse_args(argv)


def main(argv=None):
    a = parse_args(argv)
    if int(os.getenv("WORLD_SIZE", "1")) > 1:
        atorch.init_distributed("nccl" if torch.cuda.is_available() else "gloo",
                                set_cuda_device_using_local_rank=True)
    cfg = LlamaConfig.named(a.model)
    if a.num_layers:
        cfg.num_hidden_layers = a.num_layers
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, a.block_size)
    torch.manual_seed(0)
    model = Llama(cfg)
    if a.lora_rank:
        apply_lora(model, ["q_proj", "k_proj", "v_proj", "o_proj", "qkv"], rank=a.lora_rank, alpha=2 * a.lora_rank)
    args = AtorchArguments(
        output_dir=a.output_dir, per_device_train_batch_size=a.per_device_train_batch_size, max_steps=a.max_steps,
        learning_rate=a.learning_rate, lr_scheduler_type="cosine", warmup_steps=2, save_strategy="steps",
        save_steps=a.save_steps, logging_steps=a.logging_steps, bf16=a.bf16 and torch.cuda.is_available(),
        atorch_opt=a.atorch_opt if int(os.getenv("WORLD_SIZE", "1")) > 1 else "none",
        atorch_wrap_cls=(LlamaDecoderLayer,),
        atorch_checkpoint_cls=(LlamaDecoderLayer,) if a.gradient_checkpointing else None,
        model_input_format="unpack_dict", save_strategy_to_file="strategy.json", disable_tqdm=True,
        report_to=[], seed=42)
    trainer = AtorchTrainer(model=model, args=args, train_dataset=CLMDataset(cfg.vocab_size, a.block_size,
                                                                            a.samples))
    result = trainer.train(resume_from_checkpoint=True if a.resume_from_checkpoint else None)
    trainer.save_model()
    if a.lora_rank and trainer.is_world_process_zero():
        torch.save(lora_state_dict(model), os.path.join(a.output_dir, "adapter.pt"))
    if trainer.is_world_process_zero():
        print(f"global_step={trainer.state.global_step} train_loss={result.training_loss:.4f}", flush=True)
    trainer.close()
    return result


if __name__ == "__main__":
    main()
