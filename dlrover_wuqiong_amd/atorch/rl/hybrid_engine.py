"""Hybrid engine: the PPO actor generates with a KV cache from the same
weights it trains, switching from the (possibly FSDP-sharded) training
layout to an inference layout and back.

MI355X-first design (vs the reference's DeepSpeed-container swap +
optional vLLM backend):
  * ``gathered_params``: FSDP2 units are unsharded once for the whole
    rollout (one all-gather per unit over RCCL, not one per decoded token)
    and resharded before training resumes; 288 GB of HBM holds an 8B actor's
    full bf16 weights next to its shards, optimizer state and the cache;
  * a static KV cache [L, B, Smax, Hkv, D] in HBM; prefill runs the MFMA flash
    attention over the prompt and writes K/V into the cache; each decode
    step runs the split-KV decode kernel (``ops.attention.decode_attention``,
    ``csrc/kernels/attn_decode.hip``) whose lengths live on the device;
  * the decode step (embedding -> L x {RMSNorm, QKV GEMM, RoPE at the device
    positions, cache scatter, decode attention, O GEMM, RMSNorm, MLP} -> LM
    head, lengths += 1) is captured ONCE in a HIP graph and replayed per
    token, so a token costs one graph launch instead of ~15 kernel launches
    per layer.  Sampling stays outside the graph.

Works with ``models.llama.Llama`` (dense FFN for graph capture; MoE runs
eagerly), including tensor-parallel actors (each rank caches its own KV
heads, the TP layers do their own RCCL collectives, the vocab-parallel LM
head's logits are all-gathered before sampling; decoded eagerly: no graph
around collectives) and sequence-parallel actors (weights are replicated
over the SP group, so generation runs with SP switched off and every SP rank
produces the same rollout).  Parity: ATorch ``atorch/rl/ds_hybrid_engine/hybrid_engine.py``
(generate with gathered ZeRO-3 params, inference containers, KV cache) and
``rl/inference_backend/vllm_backend.py``.
"""

import contextlib
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...common.log import logger
from ...ops.attention import decode_attention, flash_attn_func
from ...ops.rope import apply_rope, rope_table


def find_llama(model: nn.Module):
    """The ``models.llama.Llama`` inside ``model`` (wrappers such as the
    autocast module of ``auto_accelerate`` or FSDP2 keep it as a submodule)."""
    from ...models.llama import Llama

    for m in model.modules():
        if isinstance(m, Llama):
            return m
    return None


@contextlib.contextmanager
def gathered_params(model: nn.Module):
    """Unshard every FSDP2 unit of ``model`` for the duration (no-op for an
    unsharded model)."""
    try:
        from torch.distributed.fsdp import FSDPModule
    except ImportError:  # pragma: no cover
        FSDPModule = ()
    units = [m for m in model.modules() if FSDPModule and isinstance(m, FSDPModule)]
    for u in units:
        u.unshard()
    try:
        yield
    finally:
        for u in units:
            u.reshard()


class KVCache:
    def __init__(self, n_layers: int, batch: int, max_len: int, n_kv: int, head_dim: int, device, dtype):
        self.k = torch.zeros(n_layers, batch, max_len, n_kv, head_dim, device=device, dtype=dtype)
        self.v = torch.zeros_like(self.k)
        self.lens = torch.zeros(batch, device=device, dtype=torch.int32)
        self.max_len = max_len

    @property
    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()


class HybridEngine:
    def __init__(self, actor: nn.Module, max_batch: int, max_len: int, use_graph: bool = True):
        self.actor = actor
        self.llama = find_llama(actor)
        if self.llama is None:
            raise TypeError("HybridEngine drives models.llama.Llama actors")
        from ...models.llama import _ws

        self.tp_group = getattr(self.llama, "tp_group", None)
        self.tp = _ws(self.tp_group)
        cfg = self.llama.cfg
        self.cfg = cfg
        self.max_batch, self.max_len = max_batch, max_len
        self.use_graph = use_graph and cfg.num_experts == 0 and self.tp == 1
        self.cache: Optional[KVCache] = None
        self._graph = None
        self._graph_key = None
        self._tok = None
        self._logits = None

    # ------------------------------------------------------------ forward
    def _ensure_cache(self, B: int, device, dtype):
        c = self.cache
        if c is None or c.k.shape[1] != B or c.k.device != device or c.k.dtype != dtype:
            cfg = self.cfg
            # this rank's KV heads (all of them without tensor parallelism)
            self.cache = KVCache(cfg.num_hidden_layers, B, self.max_len, cfg.num_key_value_heads // self.tp,
                                 cfg.head_dim, device, dtype)
            self._graph = None
            logger.info(f"hybrid engine: KV cache {self.cache.nbytes / 2**30:.2f} GiB "
                        f"({B} x {self.max_len} tokens)")
        return self.cache

    def _layer(self, li: int, layer, x, r, cos, sin, pos_ids, prefill: bool):
        attn = layer.self_attn
        if r is None:
            a, h = layer.input_layernorm(x), x
        else:
            a, h = layer.input_layernorm.add_forward(x, r)
        B, S, _ = a.shape
        qkv = attn.qkv_proj(a).view(B, S, attn.nh + 2 * attn.nkv, attn.hd)
        q, k, v = qkv.split([attn.nh, attn.nkv, attn.nkv], dim=2)
        q = apply_rope(q.contiguous(), cos, sin, pos_ids)
        k = apply_rope(k.contiguous(), cos, sin, pos_ids)
        c = self.cache
        if prefill:
            c.k[li, :B, :S] = k
            c.v[li, :B, :S] = v
            y = flash_attn_func(q, k, v.contiguous(), causal=True).reshape(B, S, attn.nh * attn.hd)
        else:
            # scatter this token's K/V at each sequence's length (device index)
            idx = (torch.arange(B, device=a.device, dtype=torch.int64) * self.max_len + c.lens.to(torch.int64))
            c.k[li].view(B * self.max_len, attn.nkv, attn.hd).index_copy_(0, idx, k.view(B, attn.nkv, attn.hd))
            c.v[li].view(B * self.max_len, attn.nkv, attn.hd).index_copy_(0, idx, v.reshape(B, attn.nkv, attn.hd))
            y = decode_attention(q.view(B, attn.nh, attn.hd), c.k[li], c.v[li], c.lens + 1)
            y = y.view(B, 1, attn.nh * attn.hd)
        b, h = layer.post_attention_layernorm.add_forward(h, attn.o_proj(y))
        return h, layer.mlp(b)

    def _forward(self, ids, prefill: bool):
        m, cfg = self.llama, self.cfg
        B, S = ids.shape
        x = m.embed_tokens(ids)
        cos, sin = rope_table(self.max_len, cfg.head_dim, cfg.rope_theta, x.device)
        pos_ids = None if prefill else self.cache.lens.view(B, 1)
        r = None
        for li, layer in enumerate(m.layers):
            x, r = self._layer(li, layer, x, r, cos, sin, pos_ids, prefill)
        x = m.norm.add_forward(x, r)[0]
        x = x[:, -1]
        logits = F.linear(x, m.embed_tokens.weight) if m.lm_head is None else m.lm_head(x)
        if self.tp > 1:
            # vocab-parallel head: every rank samples from the full vocabulary
            import torch.distributed as dist

            parts = [torch.empty_like(logits) for _ in range(self.tp)]
            dist.all_gather(parts, logits.contiguous(), group=self.tp_group)
            logits = torch.cat(parts, -1)[:, :cfg.vocab_size]
        if prefill:
            self.cache.lens.fill_(S)
        else:
            self.cache.lens.add_(1)
        return logits

    def prefill(self, prompts: torch.Tensor) -> torch.Tensor:
        B, P = prompts.shape
        if B > self.max_batch or P >= self.max_len:
            raise ValueError(f"prompts [{B}, {P}] exceed the engine ({self.max_batch}, {self.max_len})")
        dtype = self.llama.embed_tokens.weight.dtype
        self._ensure_cache(B, prompts.device, dtype)
        return self._forward(prompts, prefill=True)

    def decode(self, tok: torch.Tensor) -> torch.Tensor:
        """tok [B, 1] -> next-token logits [B, V] (graph replay when captured)."""
        if self._graph is not None:
            self._tok.copy_(tok)
            self._graph.replay()
            return self._logits
        return self._forward(tok, prefill=False)

    def _capture(self, tok: torch.Tensor):
        """Capture one decode step (the current state is not advanced:
        capture records kernels without running them)."""
        self._tok = tok.clone()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                self._logits = self._forward(self._tok, prefill=False)
        torch.cuda.current_stream().wait_stream(s)
        self._graph = g

    # ----------------------------------------------------------- generate
    @torch.no_grad()
    def generate(self, prompts: torch.Tensor, max_new_tokens: int, temperature: float = 1.0, top_k: int = 0,
                 generator: Optional[torch.Generator] = None) -> torch.Tensor:
        B, P = prompts.shape
        if P + max_new_tokens > self.max_len:
            raise ValueError(f"{P} + {max_new_tokens} tokens exceed the cache ({self.max_len})")
        was_training = self.actor.training
        self.actor.eval()
        out = [prompts]
        sp_saved = getattr(self.llama, "sp_group", None)
        if sp_saved is not None:
            self.llama.set_sp(1, 0, None)  # replicated weights: decode without the SP all-to-alls
        try:
            with gathered_params(self.actor):
                self._graph = None
                logits = self.prefill(prompts)
                for t in range(max_new_tokens):
                    nxt = _sample(logits.float(), temperature, top_k, generator)
                    if self.tp > 1:
                        # one sample per TP group: the ranks decode the same sequence
                        import torch.distributed as dist

                        dist.broadcast(nxt, dist.get_global_rank(self.tp_group, 0), group=self.tp_group)
                    out.append(nxt)
                    if t == max_new_tokens - 1:
                        break
                    if t == 0 and self.use_graph and prompts.is_cuda:
                        # one eager step (allocates every workspace), then
                        # record the step; capture does not advance the state
                        logits = self._forward(nxt, prefill=False)
                        self._capture(nxt)
                        continue
                    logits = self.decode(nxt)
                # captured against this call's weights / cache: never replayed later
                self._graph = None
        finally:
            if sp_saved is not None:
                import torch.distributed as dist

                self.llama.set_sp(dist.get_world_size(sp_saved), dist.get_rank(sp_saved), sp_saved)
            self.actor.train(was_training)
        return torch.cat(out, 1)


def _sample(logits: torch.Tensor, temperature: float, top_k: int, generator) -> torch.Tensor:
    if temperature <= 0:
        return logits.argmax(-1, keepdim=True)
    logits = logits / temperature
    if top_k:
        kth = logits.topk(top_k, dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    return torch.multinomial(logits.softmax(-1), 1, generator=generator)
