"""Shared helpers of the Llama-2 examples: synthetic token batches, FLOP
accounting and timing (reference: atorch/examples/llama2/example_utils.py)."""

import time

import torch
import torch.distributed as dist


def synthetic_batches(vocab_size: int, batch: int, seq: int, seed: int = 0):
    """Endless iterator of {"input_ids", "labels"} (labels = next tokens)."""
    g = torch.Generator().manual_seed(seed)
    while True:
        ids = torch.randint(0, vocab_size, (batch, seq + 1), generator=g)
        yield {"input_ids": ids[:, :-1], "labels": ids[:, 1:]}


def llama_train_flops(batch: int, seq: int, hidden: int, vocab: int, inter: int, layers: int,
                      act_ckpt: bool = False) -> float:
    """Model FLOPs of one training step (fwd + bwd; +1 fwd under activation
    checkpointing): QKV/O + SwiGLU MLP + causal attention + LM head."""
    per_tok_layer = 2 * (4 * hidden * hidden + 3 * hidden * inter) + 2 * seq * hidden  # causal: half of 4*S*h
    fwd = batch * seq * (layers * per_tok_layer + 2 * hidden * vocab)
    return fwd * (4 if act_ckpt else 3)


def sync_and_time() -> float:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    return time.time()


def print_rank_0(*a):
    if not dist.is_initialized() or dist.get_rank() == 0:
        print(*a, flush=True)
