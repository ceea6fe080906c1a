"""GPT-2 family on the framework's fused ops.

GPT-2 XL ("GPT2-1.5B", the reference's flash-checkpoint headline model,
docs/blogs/flash_checkpoint.md: n_layer 48, n_embd 1600) uses 25 heads of
64 (the HF configuration; the parameter count does not depend on the head
split, and head_dim 64 maps onto the MFMA attention kernel).

Hot ops: fused LayerNorm, flash attention (MFMA), fused bias+GeLU, fused
vocab cross-entropy (all HIP).  Plain GEMMs go through hipBLASLt
(``torch.nn.functional.linear``).
"""

import math
import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activation import bias_gelu
from ..ops.attention import flash_attn_qkvpacked_func
from ..ops.cross_entropy import cross_entropy
from ..ops.linear import FusedLinear, linear
from ..ops.mlp import fused_gelu_mlp
from ..ops.norm import LayerNorm

# Fused MLP (ops/mlp.py): c_fc bias in the GEMM epilogue, a GELU-only pass,
# and one pass for GELU backward + c_fc bias gradient.  With the one-pass
# backward it beats the bias-GELU kernel path on GPT2-1.5B end to end (115.6
# vs 116.3 ms/step over 2 alternations, profiles/r2/gpt2_fused_mlp_ab.txt):
# default; DWAMD_FUSED_MLP=0 selects the bias-GELU kernel path.
_FUSED_MLP = os.environ.get("DWAMD_FUSED_MLP", "1") == "1"


@dataclass
class GPT2Config:
    vocab_size: int = 50304  # 50257 padded to a multiple of 64
    n_positions: int = 1024
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    dropout: float = 0.0
    layer_norm_eps: float = 1e-5
    activation_checkpointing: bool = False

    @staticmethod
    def named(name: str) -> "GPT2Config":
        table = {
            "gpt2": dict(n_layer=12, n_head=12, n_embd=768),
            "gpt2-small": dict(n_layer=12, n_head=12, n_embd=768),
            "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),
            "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),
            "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),
            "gpt2-1.5b": dict(n_layer=48, n_head=25, n_embd=1600),
            "gpt2-tiny": dict(n_layer=2, n_head=4, n_embd=256, n_positions=256, vocab_size=1024),
        }
        return GPT2Config(**table[name.lower()])


class CausalSelfAttention(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.n_head = cfg.n_head
        self.head_dim = cfg.n_embd // cfg.n_head
        self.c_attn = FusedLinear(cfg.n_embd, 3 * cfg.n_embd)
        self.c_proj = FusedLinear(cfg.n_embd, cfg.n_embd)

    def forward(self, x):
        B, S, C = x.shape
        qkv = self.c_attn(x).view(B, S, 3, self.n_head, self.head_dim)
        y = flash_attn_qkvpacked_func(qkv, causal=True)
        return self.c_proj(y.reshape(B, S, C))


class MLP(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.c_fc = FusedLinear(cfg.n_embd, 4 * cfg.n_embd)
        self.c_proj = FusedLinear(4 * cfg.n_embd, cfg.n_embd)

    def forward(self, x):
        if type(self.c_fc) is not FusedLinear:
            # swapped projection (e.g. auto_accelerate fp8 -> Fp8Linear): its
            # own GEMM with the bias, then the activation
            return self.c_proj(bias_gelu(self.c_fc(x)))
        if _FUSED_MLP and x.is_cuda and type(self.c_proj) is FusedLinear:
            # c_fc bias in the GEMM epilogue + GELU pass; backward: c_proj
            # dgrad GEMM, then one GELU-backward + bias-gradient pass (ops/mlp.py)
            return fused_gelu_mlp(x, self.c_fc, self.c_proj)
        h = linear(x, self.c_fc.weight)  # bias fused into the activation kernel
        h = bias_gelu(h, self.c_fc.bias)
        return self.c_proj(h)


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.ln_1 = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.attn = CausalSelfAttention(cfg)
        self.ln_2 = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.mlp = MLP(cfg)

    def forward(self, x, r=None):
        """Pre-norm block on the split residual stream: the stream value is
        ``x + r`` (``r`` = previous block's MLP output, None for the first
        block), and every residual add is fused into the following norm.
        Returns ``(h, r2)`` with the block output = ``h + r2``."""
        if r is None:
            a, h = self.ln_1(x), x
        else:
            a, h = self.ln_1.add_forward(x, r)
        b, h = self.ln_2.add_forward(h, self.attn(a))
        return h, self.mlp(b)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        self.wte = nn.Embedding(cfg.vocab_size, cfg.n_embd)
        self.wpe = nn.Embedding(cfg.n_positions, cfg.n_embd)
        self.h = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.ln_f = LayerNorm(cfg.n_embd, eps=cfg.layer_norm_eps)
        self.apply(self._init)
        for n, p in self.named_parameters():
            if n.endswith("c_proj.weight"):
                nn.init.normal_(p, 0.0, 0.02 / math.sqrt(2 * cfg.n_layer))

    def init_spec(self, name: str):
        """Distribution of parameter ``name`` for sharded meta-device init
        (atorch/meta_init.py); None: by module type."""
        if name.endswith("c_proj.weight"):
            return ("normal", 0.0, 0.02 / math.sqrt(2 * self.cfg.n_layer))
        return None

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.02)
            if m.bias is not None:
                nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Embedding):
            nn.init.normal_(m.weight, 0.0, 0.02)

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def forward(self, idx, targets=None):
        B, S = idx.shape
        pos = torch.arange(S, device=idx.device)
        x = self.wte(idx) + self.wpe(pos)[None]
        r = None
        for blk in self.h:
            if self.cfg.activation_checkpointing and self.training:
                x, r = torch.utils.checkpoint.checkpoint(blk, x, r, use_reentrant=False)
            else:
                x, r = blk(x, r)
        x = self.ln_f.add_forward(x, r)[0] if r is not None else self.ln_f(x)
        logits = F.linear(x, self.wte.weight)  # tied LM head
        if targets is None:
            return logits
        return cross_entropy(logits, targets, inplace_grad=True)

    def flops_per_token(self, seq_len: int) -> float:
        """Training FLOPs/token (6N + attention)."""
        n = self.num_params() - self.wpe.weight.numel()
        c = self.cfg
        return 6 * n + 12 * c.n_layer * c.n_embd * seq_len / 2  # causal halves attention
