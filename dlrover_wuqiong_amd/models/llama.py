"""Llama family (Llama-2/3, Mistral-style GQA, Mixtral-style MoE) on the
framework's fused ops, with optional tensor / sequence / expert parallelism.

Per block: RMSNorm (HIP) -> fused QKV GEMM (hipBLASLt) -> RoPE (HIP) ->
flash attention (MFMA, GQA) -> O GEMM -> RMSNorm -> fused gate|up GEMM ->
SwiGLU (HIP) -> down GEMM; or an MoE FFN (``parallel/moe.py``).

Parallelism (all optional, orthogonal):
  * ``tp_group``: heads / FFN columns split Megatron-style
    (``parallel/tensor_parallel.py``); vocab-parallel embedding, LM head and
    cross entropy;
  * ``sp_group``: Ulysses sequence parallel -- activations are sharded along
    the sequence, one all-to-all before and after attention swaps the
    sequence and head shards;
  * ``ep_group``: expert parallel MoE FFNs.

Parity: ATorch model zoo usage of Llama (``atorch/modules/transformer``,
``examples/llama2``) and HF ``LlamaForCausalLM`` semantics (rotate-half RoPE,
RMSNorm eps, tied/untied head).
"""

import math
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.activation import swiglu
from ..ops.attention import flash_attn_func
from ..ops.cross_entropy import cross_entropy
from ..ops.norm import RMSNorm
from ..ops.rope import apply_rope, qkv_split_rope, rope_table


@dataclass
class LlamaConfig:
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    max_position_embeddings: int = 4096
    rms_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    tie_word_embeddings: bool = False
    num_experts: int = 0           # >0: MoE FFN (Mixtral-style)
    num_experts_per_tok: int = 2
    moe_intermediate_size: int = 0
    activation_checkpointing: bool = False
    head_dim_override: int = 0     # >0: head_dim != hidden/heads (e.g. one TP rank's shard)

    @property
    def head_dim(self) -> int:
        return self.head_dim_override or self.hidden_size // self.num_attention_heads

    @staticmethod
    def named(name: str) -> "LlamaConfig":
        t = {
            "llama-tiny": dict(vocab_size=1024, hidden_size=256, intermediate_size=688, num_hidden_layers=2,
                               num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512),
            "llama-moe-tiny": dict(vocab_size=1024, hidden_size=256, intermediate_size=688, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=512,
                                   num_experts=4, moe_intermediate_size=256),
            "llama2-7b": dict(),
            "llama2-13b": dict(hidden_size=5120, intermediate_size=13824, num_hidden_layers=40,
                               num_attention_heads=40, num_key_value_heads=40),
            "llama2-70b": dict(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                               num_attention_heads=64, num_key_value_heads=8),
            "llama3-8b": dict(vocab_size=128256, hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                              num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=8192,
                              rope_theta=500000.0),
            "llama3-70b": dict(vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                               num_attention_heads=64, num_key_value_heads=8, max_position_embeddings=8192,
                               rope_theta=500000.0),
            # what ONE rank of Llama-3 70B at TP=8 computes and stores (heads,
            # FFN and vocab split 8 ways; no TP collectives): checkpoint/HBM
            # sizing runs on a single GPU
            "llama3-70b-tp8-shard": dict(vocab_size=128256 // 8, hidden_size=8192, intermediate_size=28672 // 8,
                                         num_hidden_layers=80, num_attention_heads=64 // 8,
                                         num_key_value_heads=8 // 8, max_position_embeddings=8192,
                                         rope_theta=500000.0, head_dim_override=128),
            "mixtral-8x7b": dict(hidden_size=4096, intermediate_size=14336, num_hidden_layers=32,
                                 num_attention_heads=32, num_key_value_heads=8, max_position_embeddings=32768,
                                 rope_theta=1e6, num_experts=8, moe_intermediate_size=14336),
        }
        return LlamaConfig(**t[name.lower()])


def _ws(g):
    import torch.distributed as dist

    return dist.get_world_size(g) if (g is not None and dist.is_initialized()) else 1


class LlamaAttention(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_group=None, sp_group=None):
        super().__init__()
        self.cfg = cfg
        self.tp_group, self.sp_group = tp_group, sp_group
        self.cp_group = None  # context parallel (zig-zag sequence shard, K/V all-gather): Llama.set_cp
        tp = _ws(tp_group)
        assert cfg.num_attention_heads % tp == 0 and cfg.num_key_value_heads % tp == 0
        self.nh = cfg.num_attention_heads // tp
        self.nkv = cfg.num_key_value_heads // tp
        self.hd = cfg.head_dim
        qkv_out = (cfg.num_attention_heads + 2 * cfg.num_key_value_heads) * self.hd
        if tp > 1:
            from ..parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear

            self.qkv_proj = ColumnParallelLinear(cfg.hidden_size, qkv_out, bias=False, group=tp_group)
            self.o_proj = RowParallelLinear(cfg.num_attention_heads * self.hd, cfg.hidden_size, bias=False,
                                            group=tp_group)
        else:
            self.qkv_proj = nn.Linear(cfg.hidden_size, qkv_out, bias=False)
            self.o_proj = nn.Linear(cfg.num_attention_heads * self.hd, cfg.hidden_size, bias=False)

    def forward(self, x, cos, sin):
        B, S, _ = x.shape
        qkv = self.qkv_proj(x).view(B, S, self.nh + 2 * self.nkv, self.hd)
        sp = _ws(self.sp_group)
        if sp == 1:
            # one pass over the projection: split + RoPE on q, k (ops/rope.py)
            q, k, v = qkv_split_rope(qkv, self.nh, self.nkv, cos, sin)
        else:
            q, k, v = qkv.split([self.nh, self.nkv, self.nkv], dim=2)
        if sp > 1:
            from ..atorch.distributed import seq_all_to_all

            # [B, S/sp, heads, D] -> [B, S, heads/sp, D]
            q = seq_all_to_all(q.contiguous(), 2, 1, self.sp_group, sp)
            k = seq_all_to_all(k.contiguous(), 2, 1, self.sp_group, sp)
            v = seq_all_to_all(v.contiguous(), 2, 1, self.sp_group, sp)
            q = apply_rope(q.contiguous(), cos, sin)
            k = apply_rope(k.contiguous(), cos, sin)
        if self.cp_group is not None:
            from ..parallel.context_parallel import context_parallel_attention

            y = context_parallel_attention(q, k, v.contiguous(), self.cp_group, causal=True)
        else:
            y = flash_attn_func(q, k, v.contiguous(), causal=True)
        if sp > 1:
            from ..atorch.distributed import seq_all_to_all

            y = seq_all_to_all(y, 1, 2, self.sp_group, sp)
        return self.o_proj(y.reshape(B, S, self.nh * self.hd))


class LlamaMLP(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_group=None):
        super().__init__()
        tp = _ws(tp_group)
        if tp > 1:
            from ..parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear

            self.gate_up_proj = ColumnParallelLinear(cfg.hidden_size, 2 * cfg.intermediate_size, bias=False,
                                                     group=tp_group)
            self.down_proj = RowParallelLinear(cfg.intermediate_size, cfg.hidden_size, bias=False, group=tp_group)
        else:
            self.gate_up_proj = nn.Linear(cfg.hidden_size, 2 * cfg.intermediate_size, bias=False)
            self.down_proj = nn.Linear(cfg.intermediate_size, cfg.hidden_size, bias=False)

    def forward(self, x):
        return self.down_proj(swiglu(self.gate_up_proj(x)))


class LlamaDecoderLayer(nn.Module):
    def __init__(self, cfg: LlamaConfig, tp_group=None, sp_group=None, ep_group=None):
        super().__init__()
        self.input_layernorm = RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
        self.self_attn = LlamaAttention(cfg, tp_group, sp_group)
        self.post_attention_layernorm = RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
        if cfg.num_experts > 0:
            from ..parallel.moe import MoELayer

            self.mlp = MoELayer(cfg.hidden_size, cfg.moe_intermediate_size or cfg.intermediate_size,
                                cfg.num_experts, cfg.num_experts_per_tok, ep_group=ep_group)
        else:
            self.mlp = LlamaMLP(cfg, tp_group)

    def forward(self, x, cos, sin, r=None):
        """Split residual stream (value = x + r); the residual adds are fused
        into the RMSNorms.  Returns (h, mlp_out)."""
        if r is None:
            a, h = self.input_layernorm(x), x
        else:
            a, h = self.input_layernorm.add_forward(x, r)
        b, h = self.post_attention_layernorm.add_forward(h, self.self_attn(a, cos, sin))
        return h, self.mlp(b)


class Llama(nn.Module):
    """``forward(ids, targets=None)`` -> logits or mean loss.  With
    ``sp_group`` the caller passes this rank's sequence shard of ids/targets."""

    def __init__(self, cfg: LlamaConfig, tp_group=None, sp_group=None, ep_group=None):
        super().__init__()
        self.cfg = cfg
        self.tp_group, self.sp_group = tp_group, sp_group
        self.cp_group = None
        tp = _ws(tp_group)
        if tp > 1:
            from ..parallel.tensor_parallel import ColumnParallelLinear, VocabParallelEmbedding

            self.embed_tokens = VocabParallelEmbedding(cfg.vocab_size, cfg.hidden_size, group=tp_group)
            self.lm_head = ColumnParallelLinear(cfg.hidden_size, cfg.vocab_size, bias=False, group=tp_group)
        else:
            self.embed_tokens = nn.Embedding(cfg.vocab_size, cfg.hidden_size)
            self.lm_head = None if cfg.tie_word_embeddings else nn.Linear(cfg.hidden_size, cfg.vocab_size,
                                                                          bias=False)
        self.layers = nn.ModuleList([LlamaDecoderLayer(cfg, tp_group, sp_group, ep_group)
                                     for _ in range(cfg.num_hidden_layers)])
        self.norm = RMSNorm(cfg.hidden_size, eps=cfg.rms_norm_eps)
        self.apply(self._init)
        std = 0.02 / math.sqrt(2 * cfg.num_hidden_layers)
        for n, p in self.named_parameters():
            if n.endswith("o_proj.weight") or n.endswith("down_proj.weight"):
                nn.init.normal_(p, 0.0, std)

    def init_spec(self, name: str):
        """Distribution of parameter ``name`` for sharded meta-device init
        (atorch/meta_init.py); None: by module type (normal(0, 0.02) for
        Linear / Embedding, ones for norms)."""
        if name.endswith("o_proj.weight") or name.endswith("down_proj.weight"):
            return ("normal", 0.0, 0.02 / math.sqrt(2 * self.cfg.num_hidden_layers))
        return None

    @staticmethod
    def _init(m):
        if isinstance(m, nn.Linear) or type(m).__name__ in ("ColumnParallelLinear", "RowParallelLinear"):
            nn.init.normal_(m.weight, 0.0, 0.02)
        elif isinstance(m, nn.Embedding) or type(m).__name__ == "VocabParallelEmbedding":
            nn.init.normal_(m.weight, 0.0, 0.02)

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def set_sp(self, sp_size: int, sp_rank: int, sp_group):
        """Switch to Ulysses sequence parallel after construction (ATorch
        ``set_sp`` interface): forward then takes this rank's sequence shard."""
        g = sp_group if sp_size > 1 else None
        self.sp_group = g
        for layer in self.layers:
            layer.self_attn.sp_group = g

    def set_cp(self, cp_group):
        """Context parallel: forward then takes this rank's zig-zag sequence
        shard (``parallel.context_parallel.zigzag_split`` of ids/targets) and
        attends over the whole sequence; gradients are averaged over the CP
        group like data parallel."""
        g = cp_group if _ws(cp_group) > 1 else None
        self.cp_group = g
        for layer in self.layers:
            layer.self_attn.cp_group = g

    def forward(self, ids, targets=None):
        B, S = ids.shape
        sp = _ws(self.sp_group)
        x = self.embed_tokens(ids)
        if self.cp_group is not None:
            from ..parallel.context_parallel import zigzag_positions

            cp = _ws(self.cp_group)
            cos, sin = rope_table(S * cp, self.cfg.head_dim, self.cfg.rope_theta, x.device)
            pos = zigzag_positions(S, self.cp_group, device=x.device)
            cos, sin = cos[pos].contiguous(), sin[pos].contiguous()
        else:
            cos, sin = rope_table(S * sp, self.cfg.head_dim, self.cfg.rope_theta, x.device)
        r = None
        for layer in self.layers:
            if self.cfg.activation_checkpointing and self.training:
                x, r = torch.utils.checkpoint.checkpoint(layer, x, cos, sin, r, use_reentrant=False)
            else:
                x, r = layer(x, cos, sin, r)
        x = self.norm.add_forward(x, r)[0] if r is not None else self.norm(x)
        if self.lm_head is None:
            logits = F.linear(x, self.embed_tokens.weight)
        else:
            logits = self.lm_head(x)
        if targets is None:
            return logits
        if _ws(self.tp_group) > 1:
            from ..parallel.tensor_parallel import vocab_parallel_cross_entropy

            loss = vocab_parallel_cross_entropy(logits, targets, self.tp_group)
            valid = (targets != -100).sum().clamp(min=1)
            return loss.sum() / valid
        return cross_entropy(logits, targets, inplace_grad=True)

    def flops_per_token(self, seq_len: int) -> float:
        c = self.cfg
        n = self.num_params()
        return 6 * n + 12 * c.num_hidden_layers * c.hidden_size * seq_len / 2


def shard_llama_state_dict(full_sd: dict, cfg: LlamaConfig, tp_rank: int, tp: int) -> dict:
    """Slice a single-device Llama state dict for TP rank ``tp_rank`` (fused
    qkv rows regrouped per rank as [q_r | k_r | v_r], gate|up as
    [gate_r | up_r]); loads HF-converted checkpoints into a TP model."""
    if tp == 1:
        return dict(full_sd)
    hd, nh, nkv = cfg.head_dim, cfg.num_attention_heads, cfg.num_key_value_heads
    out = {}
    for k, v in full_sd.items():
        if k.endswith("qkv_proj.weight"):
            q, kk, vv = v.split([nh * hd, nkv * hd, nkv * hd], 0)
            pr = lambda t, n: t.view(n, hd, -1)[tp_rank * (n // tp):(tp_rank + 1) * (n // tp)].reshape(-1, t.shape[1])  # noqa: E731
            out[k] = torch.cat([pr(q, nh), pr(kk, nkv), pr(vv, nkv)], 0)
        elif k.endswith("gate_up_proj.weight"):
            g, u = v.chunk(2, 0)
            per = g.shape[0] // tp
            out[k] = torch.cat([g[tp_rank * per:(tp_rank + 1) * per], u[tp_rank * per:(tp_rank + 1) * per]], 0)
        elif k.endswith("o_proj.weight") or k.endswith("down_proj.weight"):
            per = v.shape[1] // tp
            out[k] = v[:, tp_rank * per:(tp_rank + 1) * per]
        elif k.endswith("embed_tokens.weight") or k.endswith("lm_head.weight"):
            per = (v.shape[0] + tp - 1) // tp
            part = v[tp_rank * per:(tp_rank + 1) * per]
            if part.shape[0] < per:
                part = torch.cat([part, part.new_zeros(per - part.shape[0], part.shape[1])], 0)
            out[k] = part
        else:
            out[k] = v
    return {k: v.contiguous() for k, v in out.items()}
