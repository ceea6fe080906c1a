"""Pipeline parallelism: stage partitioning + GPipe / 1F1B / interleaved-1F1B
schedules over point-to-point RCCL (gloo on CPU).

Reference parity: ATorch's pipeline strategy compiles a model into PiPPy
stages and runs them with torch RPC drivers
(``atorch/auto/opt_lib/pipeline_parallel_optimization.py``,
``atorch/modules/distributed_modules/compilers/pipe_compiler/PipelineStage.py``,
``distributed_pippy_compiler.py``) or DeepSpeed's ``PipelineModule``
(``atorch/utils/ds_pipe_utils.py``, ``auto/opt_lib/ds_3d_parallel_optimization.py``).
This module is the framework's own design, not a tracer:

* a model is split at decoder-layer boundaries (``split_model``) into a
  ``PipelineStage`` whose forward maps a tuple of activations to a tuple of
  activations (the first stage takes token ids, the last returns the loss);
  layers are balanced by a cost model that charges the embedding and the LM
  head + vocab cross-entropy in layer equivalents;
* activations move between neighbouring stages with batched
  ``isend``/``irecv`` (one RCCL group call per exchange, so the steady-state
  "send activation / receive gradient" pair never deadlocks); on an MI355X
  node each neighbour pair has a direct xGMI link, so a stage boundary costs
  one link's bandwidth -- place PP across nodes and TP inside the node
  (``parallel/state.py`` rank order tp -> cp -> dp -> pp);
* the schedules are host-side loops over the stage (no RPC driver process):
  ``gpipe`` (all forwards, then all backwards), ``1f1b`` (PipeDream-flush:
  ``pp - stage - 1`` warm-up forwards, steady one-forward-one-backward,
  cool-down) and ``interleaved`` (Megatron-style virtual stages: each rank
  owns ``v`` model chunks, shrinking the bubble by ``v``);
* every stage boundary carries the split residual stream ``(x, r)`` of
  shape ``(micro_batch, seq, hidden)``; the first stage broadcasts the batch
  shape over the pipeline group once per step, so every rank sizes its
  receive buffers itself (the sequence length may change between steps);
* data-parallel gradient all-reduce (``FlatDDP``) fires only on the last
  micro-batch's backward, so it overlaps the pipeline cool-down; tied input
  embedding / LM head gradients are summed over the first+last stage group.
"""

from typing import List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
import torch.nn as nn

Tensors = Tuple[torch.Tensor, ...]



# ----------------------------------------------------------------------------- partitioning


def partition_layers(num_layers: int, num_stages: int, embed_cost: float = 0.0, head_cost: float = 0.0,
                     layer_costs: Optional[Sequence[float]] = None) -> List[Tuple[int, int]]:
    """Split ``num_layers`` decoder layers into ``num_stages`` contiguous
    ranges minimising the maximum stage cost (every stage gets >= 1 layer).
    ``embed_cost`` / ``head_cost`` (layer equivalents) are charged to the
    first / last stage.  Exact DP over split points (O(L^2 * P), L <= a few
    hundred)."""
    if num_stages < 1 or num_layers < num_stages:
        raise ValueError(f"cannot split {num_layers} layers into {num_stages} stages")
    costs = list(layer_costs) if layer_costs is not None else [1.0] * num_layers
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)

    def cost(s, a, b):
        v = pre[b] - pre[a]
        if s == 0:
            v += embed_cost
        if s == num_stages - 1:
            v += head_cost
        return v

    INF = float("inf")
    # best[s][b] = min over splits of max stage cost for stages 0..s covering layers [0, b)
    best = [[INF] * (num_layers + 1) for _ in range(num_stages)]
    arg = [[0] * (num_layers + 1) for _ in range(num_stages)]
    for b in range(1, num_layers + 1):
        best[0][b] = cost(0, 0, b)
    for s in range(1, num_stages):
        for b in range(s + 1, num_layers + 1):
            for a in range(s, b):
                v = max(best[s - 1][a], cost(s, a, b))
                if v < best[s][b]:
                    best[s][b], arg[s][b] = v, a
    bounds, b = [], num_layers
    for s in range(num_stages - 1, 0, -1):
        a = arg[s][b]
        bounds.append((a, b))
        b = a
    bounds.append((0, b))
    return bounds[::-1]


class PipelineStage(nn.Module):
    """Base class: ``forward(*acts, targets=None)``.  First stage: ``acts`` =
    (token ids,).  Middle stages return a tuple of activations.  The last
    stage returns the mean loss (given targets) or the logits."""

    is_first: bool = True
    is_last: bool = True

    def tied_parameters(self) -> List[nn.Parameter]:
        """Parameters replicated on the first and last stage (tied input
        embedding / LM head); their gradients are summed across the two."""
        return []

    def act_meta(self, micro_batch: int, seq: int) -> List[Tuple[torch.dtype, Tuple[int, ...]]]:
        """(dtype, shape) of every tensor crossing a stage boundary."""
        dt = next(p.dtype for p in self.parameters() if p.is_floating_point())
        return [(dt, (micro_batch, seq, self.hidden))] * 2


class GPT2Stage(PipelineStage):
    def __init__(self, model, start: int, end: int, is_first: bool, is_last: bool):
        super().__init__()
        self.cfg = model.cfg
        self.hidden = model.cfg.n_embd
        self.is_first, self.is_last = is_first, is_last
        self.start, self.end = start, end
        self.h = nn.ModuleList(list(model.h[start:end]))
        if is_first:
            self.wte, self.wpe = model.wte, model.wpe
        if is_last:
            self.ln_f = model.ln_f
            if not is_first:
                # own copy of the tied LM-head weight, kept identical to the
                # first stage's embedding (broadcast at setup, grads summed)
                self.head_weight = nn.Parameter(model.wte.weight.detach().clone())

    def _head_w(self):
        return self.wte.weight if self.is_first else self.head_weight

    def tied_parameters(self):
        if self.is_first and self.is_last:
            return []
        if self.is_first:
            return [self.wte.weight]
        if self.is_last:
            return [self.head_weight]
        return []

    def forward(self, *acts, targets=None):
        import torch.nn.functional as F

        from ..ops.cross_entropy import cross_entropy

        if self.is_first:
            idx = acts[0]
            pos = torch.arange(idx.shape[1], device=idx.device)
            x, r = self.wte(idx) + self.wpe(pos)[None], None
        else:
            x, r = acts
        for blk in self.h:
            if self.cfg.activation_checkpointing and self.training:
                x, r = torch.utils.checkpoint.checkpoint(blk, x, r, use_reentrant=False)
            else:
                x, r = blk(x, r)
        if not self.is_last:
            return x, r
        x = self.ln_f.add_forward(x, r)[0]
        logits = F.linear(x, self._head_w())
        if targets is None:
            return logits
        return cross_entropy(logits, targets, inplace_grad=True)


class LlamaStage(PipelineStage):
    def __init__(self, model, start: int, end: int, is_first: bool, is_last: bool):
        super().__init__()
        self.cfg = model.cfg
        self.tp_group = model.tp_group
        self.hidden = model.cfg.hidden_size
        self.is_first, self.is_last = is_first, is_last
        self.start, self.end = start, end
        self.layers = nn.ModuleList(list(model.layers[start:end]))
        if is_first:
            self.embed_tokens = model.embed_tokens
        if is_last:
            self.norm = model.norm
            if model.lm_head is not None:
                self.lm_head = model.lm_head
            else:
                self.lm_head = None
            if model.lm_head is None and not is_first:
                self.head_weight = nn.Parameter(model.embed_tokens.weight.detach().clone())

    def tied_parameters(self):
        if not self.cfg.tie_word_embeddings or (self.is_first and self.is_last):
            return []
        if self.is_first:
            return [self.embed_tokens.weight]
        if self.is_last:
            return [self.head_weight]
        return []

    def forward(self, *acts, targets=None):
        import torch.nn.functional as F

        from ..models.llama import rope_table
        from ..ops.cross_entropy import cross_entropy

        if self.is_first:
            x, r = self.embed_tokens(acts[0]), None
        else:
            x, r = acts
        cos, sin = rope_table(x.shape[1], self.cfg.head_dim, self.cfg.rope_theta, x.device)
        for layer in self.layers:
            if self.cfg.activation_checkpointing and self.training:
                x, r = torch.utils.checkpoint.checkpoint(layer, x, cos, sin, r, use_reentrant=False)
            else:
                x, r = layer(x, cos, sin, r)
        if not self.is_last:
            return x, r
        x = self.norm.add_forward(x, r)[0]
        if self.lm_head is not None:
            logits = self.lm_head(x)
        else:
            logits = F.linear(x, self.embed_tokens.weight if self.is_first else self.head_weight)
        if targets is None:
            return logits
        if self.tp_group is not None and dist.get_world_size(self.tp_group) > 1:
            from .tensor_parallel import vocab_parallel_cross_entropy

            loss = vocab_parallel_cross_entropy(logits, targets, self.tp_group)
            return loss.sum() / (targets != -100).sum().clamp(min=1)
        return cross_entropy(logits, targets, inplace_grad=True)


class DecoderParts:
    """The pieces of a generic decoder-only LM (any transformers causal LM --
    Llama, Qwen2, Mistral, GPT-NeoX, GPT-2, Phi ... -- or a user model of
    the same shape), found structurally rather than by class:

    * ``layers``: the longest ``nn.ModuleList`` of same-class blocks that
      hold parameters (the decoder layers); its parent is the backbone;
    * ``embed``: the backbone's token ``nn.Embedding`` (vocabulary-sized, or
      the first Embedding registered before the layers); ``pos_embed``: a
      second Embedding before the layers (learned positions, GPT-2);
      ``drop``: a Dropout registered before the layers;
    * ``norm``: the first module registered after the layers;
    * ``rotary``: a backbone child whose class name mentions "Rotary"
      (``forward(x, position_ids) -> (cos, sin)``);
    * ``head``: the top-level ``nn.Linear`` producing vocabulary logits
      (tied when its weight IS the embedding's)."""

    def __init__(self, model: nn.Module):
        lists = [(n, m) for n, m in model.named_modules() if isinstance(m, nn.ModuleList) and len(m) > 0
                 and len({type(x) for x in m}) == 1 and any(True for _ in m[0].parameters())]
        if not lists:
            raise TypeError(f"no decoder layer stack found in {type(model).__name__}")
        lname, layers = max(lists, key=lambda x: len(x[1]))
        self.layers = layers
        bname = lname.rsplit(".", 1)[0] if "." in lname else ""
        self.backbone = model.get_submodule(bname) if bname else model
        self.config = getattr(model, "config", None) or getattr(self.backbone, "config", None)
        kids = list(self.backbone.named_children())
        li = next(i for i, (_n, m) in enumerate(kids) if m is layers)
        before, after = kids[:li], kids[li + 1:]
        vocab = getattr(self.config, "vocab_size", None)
        embs = [m for _n, m in before if isinstance(m, nn.Embedding)]
        if not embs:
            raise TypeError(f"{type(model).__name__}: no token embedding before the decoder layers")
        tok = [m for m in embs if vocab is not None and m.num_embeddings == vocab]
        self.embed = tok[0] if tok else embs[0]
        others = [m for m in embs if m is not self.embed]
        self.pos_embed = others[0] if others else None
        drops = [m for _n, m in before if isinstance(m, nn.Dropout)]
        self.drop = drops[0] if drops else None
        norms = [m for _n, m in after if "rotary" not in type(m).__name__.lower()]
        self.norm = norms[0] if norms else None
        rot = [m for _n, m in kids if "rotary" in type(m).__name__.lower()]
        self.rotary = rot[0] if rot else None
        heads = [m for _n, m in model.named_children() if isinstance(m, nn.Linear)
                 and (vocab is None or m.out_features == vocab)]
        if not heads:
            raise TypeError(f"{type(model).__name__}: no LM head (Linear to the vocabulary) at the top level")
        self.head = heads[0]
        self.tied = self.head.weight is self.embed.weight
        self.hidden = self.embed.embedding_dim
        self.vocab = self.head.out_features
        if self.config is not None and getattr(self.config, "_attn_implementation", None) == "eager":
            # eager attention needs an explicit causal mask; sdpa / flash
            # take attention_mask=None as causal
            self.config._attn_implementation = "sdpa"


class DecoderStackStage(PipelineStage):
    """A contiguous range of decoder layers of any :class:`DecoderParts`
    model.  One tensor crosses each boundary: the hidden states."""

    def __init__(self, parts: DecoderParts, start: int, end: int, is_first: bool, is_last: bool):
        super().__init__()
        self.parts_cfg = parts.config
        self.hidden = parts.hidden
        self.is_first, self.is_last = is_first, is_last
        self.start, self.end = start, end
        self.layers = nn.ModuleList(list(parts.layers[start:end]))
        self.rotary = parts.rotary
        self.tied = parts.tied
        if is_first:
            self.embed = parts.embed
            self.pos_embed = parts.pos_embed
            self.drop = parts.drop
        if is_last:
            self.norm = parts.norm
            if parts.tied and not is_first:
                self.head_weight = nn.Parameter(parts.embed.weight.detach().clone())
            elif not parts.tied:
                self.head = parts.head

    def tied_parameters(self):
        if not self.tied or (self.is_first and self.is_last):
            return []
        if self.is_first:
            return [self.embed.weight]
        if self.is_last:
            return [self.head_weight]
        return []

    def act_meta(self, micro_batch: int, seq: int):
        dt = next(p.dtype for p in self.parameters() if p.is_floating_point())
        return [(dt, (micro_batch, seq, self.hidden))]

    def _masks(self, x, pos):
        cfg = self.parts_cfg
        try:
            from transformers.masking_utils import create_causal_mask, create_sliding_window_causal_mask
        except Exception:
            return {"full_attention": None}
        kw = dict(config=cfg, inputs_embeds=x, attention_mask=None, past_key_values=None, position_ids=pos)
        if self._uniform_sliding():
            # Mistral-style: no per-layer types, every layer uses the window
            # when the config sets one (MistralModel.forward's mask choice)
            return {"sliding_attention": create_sliding_window_causal_mask(**kw)}
        out = {"full_attention": create_causal_mask(**kw)}
        if "sliding_attention" in (getattr(cfg, "layer_types", None) or []):
            out["sliding_attention"] = create_sliding_window_causal_mask(**kw)
        return out

    def _uniform_sliding(self) -> bool:
        cfg = self.parts_cfg
        return (cfg is not None and not getattr(cfg, "layer_types", None)
                and getattr(cfg, "sliding_window", None) is not None)

    def forward(self, *acts, targets=None):
        import torch.nn.functional as F

        from ..ops.cross_entropy import cross_entropy

        if self.is_first:
            ids = acts[0]
            x = self.embed(ids)
            if self.pos_embed is not None:
                x = x + self.pos_embed(torch.arange(ids.shape[1], device=ids.device))[None]
            if self.drop is not None:
                x = self.drop(x)
        else:
            x = acts[0]
        pos = torch.arange(x.shape[1], device=x.device)[None]
        masks = self._masks(x, pos) if self.parts_cfg is not None else {"full_attention": None}
        kw = {"position_ids": pos}
        if self.rotary is not None:
            kw["position_embeddings"] = self.rotary(x, pos)
        types = getattr(self.parts_cfg, "layer_types", None)
        default_t = "sliding_attention" if self._uniform_sliding() else "full_attention"
        for i, layer in enumerate(self.layers):
            t = types[self.start + i] if types else default_t
            out = layer(x, attention_mask=masks.get(t), **kw)
            x = out[0] if isinstance(out, (tuple, list)) else out
        if not self.is_last:
            return (x,)
        if self.norm is not None:
            x = self.norm(x)
        if self.tied:
            logits = F.linear(x, self.embed.weight if self.is_first else self.head_weight)
        else:
            logits = self.head(x)
        if hasattr(logits, "to_local"):  # a DTensor-parallel head
            logits = logits.full_tensor()
        if targets is None:
            return logits
        return cross_entropy(logits, targets, inplace_grad=True)


class SequentialStage(PipelineStage):
    """A contiguous range of an ``nn.Sequential`` (one tensor between
    children); the last stage applies ``loss_fn(output, targets)``."""

    def __init__(self, seq: nn.Sequential, start: int, end: int, is_first: bool, is_last: bool, loss_fn=None,
                 boundary_shape=None):
        super().__init__()
        self.body = nn.Sequential(*list(seq)[start:end])
        self.is_first, self.is_last = is_first, is_last
        self.loss_fn = loss_fn
        self.boundary_shape = boundary_shape  # fn(micro_batch, seq) -> (dtype, shape)

    def act_meta(self, micro_batch: int, seq: int):
        if self.boundary_shape is None:
            raise ValueError("SequentialStage needs boundary_shape(micro_batch, seq) -> (dtype, shape)")
        return [self.boundary_shape(micro_batch, seq)]

    def forward(self, *acts, targets=None):
        y = self.body(acts[0])
        if not self.is_last:
            return (y,)
        if targets is None or self.loss_fn is None:
            return y
        return self.loss_fn(y, targets)


def split_model(model: nn.Module, num_stages: int, stage: int, bounds: Optional[List[Tuple[int, int]]] = None,
                virtual_chunk: Optional[Tuple[int, int]] = None, **kw) -> PipelineStage:
    """Cut a model at decoder-layer boundaries and return the piece for
    pipeline ``stage``: this package's GPT-2 / Llama, any decoder-only LM
    whose layer stack :class:`DecoderParts` finds (transformers Qwen2,
    Mistral, GPT-NeoX, GPT-2, Llama ...), or an ``nn.Sequential`` (cut
    between children; pass ``loss_fn`` and ``boundary_shape``).  With
    ``virtual_chunk=(chunk, v)`` the layers are cut into ``num_stages * v``
    pieces and piece ``chunk * num_stages + stage`` is returned
    (interleaved schedule)."""
    from ..models.gpt2 import GPT2
    from ..models.llama import Llama

    if isinstance(model, GPT2):
        n, cls = model.cfg.n_layer, GPT2Stage
        vocab, hidden = model.cfg.vocab_size, model.cfg.n_embd
    elif isinstance(model, Llama):
        n, cls = model.cfg.num_hidden_layers, LlamaStage
        vocab, hidden = model.cfg.vocab_size, model.cfg.hidden_size
    elif isinstance(model, nn.Sequential):
        chunks, piece = num_stages, stage
        if virtual_chunk is not None:
            c, v = virtual_chunk
            chunks, piece = num_stages * v, c * num_stages + stage
        a, b = (bounds or partition_layers(len(model), chunks))[piece]
        return SequentialStage(model, a, b, is_first=(piece == 0), is_last=(piece == chunks - 1),
                               loss_fn=kw.get("loss_fn"), boundary_shape=kw.get("boundary_shape"))
    else:
        parts = DecoderParts(model)
        n, vocab, hidden = len(parts.layers), parts.vocab, parts.hidden

        def cls(_m, a, b, is_first, is_last):
            return DecoderStackStage(parts, a, b, is_first, is_last)
    chunks, piece = num_stages, stage
    if virtual_chunk is not None:
        c, v = virtual_chunk
        chunks, piece = num_stages * v, c * num_stages + stage
    if bounds is None:
        # LM head GEMM + vocab cross-entropy ~ vocab / (12 * hidden) layers
        head = vocab / (12.0 * hidden) + 0.2
        bounds = partition_layers(n, chunks, embed_cost=0.1, head_cost=head)
    a, b = bounds[piece]
    return cls(model, a, b, is_first=(piece == 0), is_last=(piece == chunks - 1))




# ----------------------------------------------------------------------------- schedules


class PipelineSchedule:
    """Run one training step of a pipelined model on this rank.

    ``stages``: this rank's ``PipelineStage``, or a list of ``v`` chunks for
    the interleaved schedule (chunk ``c`` = global piece ``c * pp + rank``,
    see ``build_pipeline``).  ``step(ids, targets)`` splits the local batch
    into ``num_microbatches`` along dim 0, runs every forward/backward and
    returns the mean loss (broadcast from the last stage to the whole
    pipeline group).  Gradients accumulate into the parameters' ``.grad``;
    run the optimizer afterwards.  ``ids`` is only read on the first stage
    and ``targets`` only on the last.
    """

    def __init__(self, stages: Union[PipelineStage, Sequence[PipelineStage]], num_microbatches: int,
                 group=None, schedule: str = "1f1b", ddp=None, embedding_group=None,
                 device: Optional[torch.device] = None, broadcast_loss: bool = True):
        self.chunks = list(stages) if isinstance(stages, (list, tuple)) else [stages]
        self.v = len(self.chunks)
        self.M = num_microbatches
        self.group = group
        self.schedule = "interleaved" if self.v > 1 else schedule
        if self.schedule not in ("gpipe", "1f1b", "interleaved"):
            raise ValueError(f"unknown schedule {schedule}")
        self.P = (dist.get_world_size(group) if dist.is_initialized() else 1)
        if self.P > 1:
            ranks = dist.get_process_group_ranks(group) if group is not None else list(range(self.P))
            me = dist.get_rank()
            self.ranks = ranks
            self.s = ranks.index(me)
            self.prev_rank = ranks[(self.s - 1) % self.P]
            self.next_rank = ranks[(self.s + 1) % self.P]
        else:
            self.ranks, self.s = [0], 0
        if self.v > 1 and num_microbatches % self.P != 0:
            raise ValueError("interleaved schedule needs num_microbatches % pp == 0")
        self.ddp = ddp
        self.embedding_group = embedding_group
        self.broadcast_loss = broadcast_loss
        p = next(self.chunks[0].parameters(), None)
        self.device = device or (p.device if p is not None else torch.device("cpu"))
        self.bytes_sent = 0
        if self.P > 1:
            self._sync_tied_weights()

    # -- tied weights ------------------------------------------------------------
    def _tied(self):
        out = []
        for c in self.chunks:
            out += c.tied_parameters()
        return out

    def _sync_tied_weights(self):
        tied = self._tied()
        if tied and self.embedding_group is not None:
            src = min(dist.get_process_group_ranks(self.embedding_group))
            for p in tied:
                dist.broadcast(p.data, src=src, group=self.embedding_group)

    def _reduce_tied_grads(self):
        tied = self._tied()
        if tied and self.embedding_group is not None:
            for p in tied:
                if p.grad is not None:
                    dist.all_reduce(p.grad, group=self.embedding_group)

    # -- communication -------------------------------------------------------------
    def _comm(self, send_next: Optional[Tensors] = None, send_prev: Optional[Tensors] = None,
              recv_prev: bool = False, recv_next: bool = False):
        """One batched neighbour exchange (a single RCCL group call).  Sends
        go downstream (activations, tag 1) / upstream (gradients, tag 2);
        receives are posted in the same order so that message matching per
        peer is unambiguous even when prev == next (pp == 2)."""
        if self.P == 1:
            return None, None
        ops = []
        if send_next is not None:
            for t in send_next:
                t = t.contiguous()
                self.bytes_sent += t.numel() * t.element_size()
                ops.append(dist.P2POp(dist.isend, t, self.next_rank, self.group, 1))
        if send_prev is not None:
            for t in send_prev:
                t = t.contiguous()
                self.bytes_sent += t.numel() * t.element_size()
                ops.append(dist.P2POp(dist.isend, t, self.prev_rank, self.group, 2))
        fwd = bwd = None
        if recv_prev:
            fwd = tuple(torch.empty(sh, dtype=dt, device=self.device) for dt, sh in self.meta)
            ops += [dist.P2POp(dist.irecv, b, self.prev_rank, self.group, 1) for b in fwd]
        if recv_next:
            bwd = tuple(torch.empty(sh, dtype=dt, device=self.device) for dt, sh in self.meta)
            ops += [dist.P2POp(dist.irecv, b, self.next_rank, self.group, 2) for b in bwd]
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return fwd, bwd

    # -- compute -----------------------------------------------------------------
    def _forward(self, c: int, acts: Optional[Tensors]) -> Tensors:
        st = self.chunks[c]
        mb = self._fcount[c]
        self._fcount[c] += 1
        if st.is_first:
            inp = (self._ids[mb],)
        else:
            inp = tuple(a.detach().requires_grad_(a.is_floating_point()) for a in acts)
        if st.is_last:
            loss = st(*inp, targets=self._tgt[mb])
            self._losses.append(loss.detach())
            out = (loss / self.M,)
        else:
            out = _as_tuple(st(*inp))
        self._store[c].append((inp, out))
        return out

    def _backward(self, c: int, grads: Optional[Tensors]) -> Optional[Tensors]:
        st = self.chunks[c]
        if self.ddp is not None:
            # data-parallel buckets launch only on each chunk's last micro-batch
            self.ddp._sync = self._bcount[c] == self.M - 1
        self._bcount[c] += 1
        inputs, outputs = self._store[c].pop(0)
        if st.is_last:
            torch.autograd.backward(outputs[0])
        else:
            pairs = [(o, g) for o, g in zip(outputs, grads) if o.requires_grad]
            torch.autograd.backward([o for o, _ in pairs], grad_tensors=[g for _, g in pairs])
        if st.is_first:
            return None
        return tuple(i.grad if i.grad is not None else torch.zeros_like(i) for i in inputs)

    # -- public --------------------------------------------------------------------
    def step(self, ids: Optional[torch.Tensor], targets: Optional[torch.Tensor]) -> torch.Tensor:
        M = self.M
        shape = torch.tensor(list(ids.shape) if ids is not None else [0, 0], dtype=torch.int64, device=self.device)
        if self.P > 1:
            dist.broadcast(shape, src=self.ranks[0], group=self.group)
        B, S = (int(x) for x in shape.tolist())
        if B % M != 0:
            raise ValueError(f"batch of {B} cannot be split into {M} micro-batches")
        self.meta = self.chunks[0].act_meta(B // M, S)
        self._ids = ids.chunk(M, dim=0) if ids is not None else None
        self._tgt = targets.chunk(M, dim=0) if targets is not None else None
        self._store = [[] for _ in self.chunks]
        self._fcount = [0] * self.v
        self._bcount = [0] * self.v
        self._losses = []
        if self.ddp is not None:
            self.ddp._reset()
        try:
            if self.schedule == "gpipe":
                self._run_gpipe()
            elif self.schedule == "1f1b":
                self._run_1f1b()
            else:
                self._run_interleaved()
        finally:
            if self.ddp is not None:
                self.ddp._sync = True
        self._reduce_tied_grads()
        if self.ddp is not None:
            self.ddp.finish_gradient_sync()
        loss = torch.stack(self._losses).mean().float() if self._losses else torch.zeros((), device=self.device)
        self._ids = self._tgt = None
        if self.broadcast_loss and self.P > 1:
            loss = loss.reshape(1).clone()
            dist.broadcast(loss, src=self.ranks[-1], group=self.group)
            loss = loss[0]
        return loss

    # -- GPipe -----------------------------------------------------------------------
    def _run_gpipe(self):
        st = self.chunks[0]
        outs = []
        for _ in range(self.M):
            acts, _ = self._comm(recv_prev=not st.is_first)
            out = self._forward(0, acts)
            self._comm(send_next=None if st.is_last else out)
            outs.append(out)
        for _ in range(self.M):
            _, g = self._comm(recv_next=not st.is_last)
            dx = self._backward(0, g)
            self._comm(send_prev=dx)

    # -- 1F1B (PipeDream-flush) ---------------------------------------------------------
    def _run_1f1b(self):
        st = self.chunks[0]
        M, P, s = self.M, self.P, self.s
        warm = min(P - s - 1, M)
        rem = M - warm
        for _ in range(warm):
            acts, _ = self._comm(recv_prev=not st.is_first)
            out = self._forward(0, acts)
            self._comm(send_next=None if st.is_last else out)
        acts = self._comm(recv_prev=not st.is_first)[0] if rem > 0 else None
        for i in range(rem):
            out = self._forward(0, acts)
            _, g = self._comm(send_next=None if st.is_last else out, recv_next=not st.is_last)
            dx = self._backward(0, g)
            last = i == rem - 1
            acts, _ = self._comm(send_prev=dx, recv_prev=(not last) and not st.is_first)
        for _ in range(warm):
            _, g = self._comm(recv_next=not st.is_last)
            dx = self._backward(0, g)
            self._comm(send_prev=dx)

    # -- interleaved 1F1B (virtual pipeline) ------------------------------------------------
    def _run_interleaved(self):
        """Megatron's interleaved schedule.  Virtual step k runs chunk
        ``(k % (P*v)) // P`` (forward; reversed for backward).  Piece c of
        the last rank feeds piece c+1 of rank 0 (the pipeline ring wraps), so
        every transfer stays a neighbour exchange, and each exchange pairs the
        sends and receives of one step in a single group call."""
        P, s, v, M = self.P, self.s, self.v, self.M
        total = M * v

        def chunk(k, fwd=True):
            c = (k % (P * v)) // P
            return c if fwd else v - 1 - c

        def is_first(c):
            return self.chunks[c].is_first

        def is_last(c):
            return self.chunks[c].is_last

        in_q: List[list] = [[] for _ in range(v)]
        g_q: List[list] = [[] for _ in range(v)]

        def fwd_step(k):
            c = chunk(k, True)
            acts = None if is_first(c) else in_q[c].pop(0)
            return c, self._forward(c, acts)

        def bwd_step(k):
            c = chunk(k, False)
            g = None if is_last(c) else g_q[c].pop(0)
            return c, self._backward(c, g)

        if M == P:
            warm, all_warm = total, True
        else:
            warm = (P - s - 1) * 2 + (v - 1) * P
            all_warm = warm >= total
            warm = min(warm, total)
        rem = total - warm

        if not is_first(0):
            in_q[0].append(self._comm(recv_prev=True)[0])
        for k in range(warm):
            c, out = fwd_step(k)
            nf = chunk(k + 1, True)
            recv_prev = not (s == 0 and nf == 0) and k != total - 1
            send = None if is_last(c) else out
            if k == warm - 1 and not all_warm:
                recv_next = s != P - 1
                x, g = self._comm(send_next=send, recv_prev=recv_prev, recv_next=recv_next)
                if recv_next:
                    g_q[v - 1].append(g)
            else:
                x, _ = self._comm(send_next=send, recv_prev=recv_prev)
            if recv_prev:
                in_q[nf].append(x)

        for k in range(rem):
            fk = k + warm
            fc, out = fwd_step(fk)
            bc, dx = bwd_step(k)
            send_f = None if is_last(fc) else out
            send_b = None if is_first(bc) else dx
            recv_prev = True
            if s == 0:
                nf = chunk(fk - (P - 1), True)
                if nf == v - 1:
                    recv_prev = False
                nf += 1
            else:
                nf = chunk(fk + 1, True)
            recv_next = True
            if s == P - 1:
                nb = chunk(k - (P - 1), False)
                if nb == 0:
                    recv_next = False
                nb -= 1
            else:
                nb = chunk(k + 1, False)
            if k == rem - 1:
                recv_prev = False
            x, g = self._comm(send_next=send_f, send_prev=send_b, recv_prev=recv_prev, recv_next=recv_next)
            if recv_prev:
                in_q[nf].append(x)
            if recv_next:
                g_q[nb].append(g)

        if all_warm and s != P - 1:
            g_q[v - 1].append(self._comm(recv_next=True)[1])
        for k in range(rem, total):
            bc, dx = bwd_step(k)
            nb = chunk(k + 1, False)
            recv_next = not (s == P - 1 and nb == v - 1) and k != total - 1
            _, g = self._comm(send_prev=None if is_first(bc) else dx, recv_next=recv_next)
            if recv_next:
                g_q[nb].append(g)


def _as_tuple(x) -> Tensors:
    if isinstance(x, torch.Tensor):
        return (x,)
    return tuple(x)


def build_pipeline(model: nn.Module, num_stages: int, stage: int, virtual_stages: int = 1,
                   bounds: Optional[List[Tuple[int, int]]] = None, **kw) -> Union[PipelineStage, List[PipelineStage]]:
    """This rank's stage (or its ``virtual_stages`` interleaved chunks)."""
    if virtual_stages == 1:
        return split_model(model, num_stages, stage, bounds, **kw)
    return [split_model(model, num_stages, stage, bounds, virtual_chunk=(c, virtual_stages), **kw)
            for c in range(virtual_stages)]


class PipelineModule(nn.Module):
    """Holds this rank's chunks in one module (so ``FlatParams`` / an
    optimizer / a checkpointer see one parameter set) and exposes the
    schedule: ``loss = pipe.train_step(ids, targets)``."""

    def __init__(self, model: nn.Module, num_stages: int, stage: int, num_microbatches: int,
                 schedule: str = "1f1b", virtual_stages: int = 1, group=None, embedding_group=None,
                 bounds: Optional[List[Tuple[int, int]]] = None, **split_kw):
        super().__init__()
        chunks = build_pipeline(model, num_stages, stage, virtual_stages, bounds, **split_kw)
        self.chunks = nn.ModuleList(chunks if isinstance(chunks, list) else [chunks])
        self.num_stages, self.stage = num_stages, stage
        self.num_microbatches = num_microbatches
        self.schedule_name = schedule
        self.group, self.embedding_group = group, embedding_group
        self._schedule: Optional[PipelineSchedule] = None
        self.ddp = None  # FlatDDP over the data-parallel group (flat buffers)
        self.dp_group = None  # or: plain gradient all-reduce over this group after each step
        self.amp_dtype = None

    def schedule(self) -> PipelineSchedule:
        if self._schedule is None:
            self._schedule = PipelineSchedule(list(self.chunks), self.num_microbatches, group=self.group,
                                              schedule=self.schedule_name, ddp=self.ddp,
                                              embedding_group=self.embedding_group)
        return self._schedule

    def train_step(self, ids, targets):
        if self.amp_dtype is not None:
            with torch.autocast("cuda" if torch.cuda.is_available() else "cpu", dtype=self.amp_dtype):
                loss = self.schedule().step(ids, targets)
        else:
            loss = self.schedule().step(ids, targets)
        if self.dp_group is not None and self.ddp is None:
            self._allreduce_dp_grads()
        return loss

    def train_batch(self, data_iter):
        """DeepSpeed-engine style step (reference ds_3d_llama2.py:
        ``loss = model.train_batch(data_iter)``): pulls ``num_microbatches``
        micro-batches, maps each through ``batch_fn`` (default: a dict's
        ``input_ids`` / ``labels``, or an ``(ids, targets)`` pair; a
        ``((ids, ...), (targets, ...))`` result keeps the first of each) and
        runs one pipeline step over their concatenation."""
        ids, tgts = [], []
        for _ in range(self.num_microbatches):
            i, t = self._split_batch(next(data_iter))
            ids.append(i)
            tgts.append(t)
        return self.train_step(torch.cat(ids), torch.cat(tgts))

    def _split_batch(self, data):
        fn = getattr(self, "batch_fn", None)
        if fn is not None:
            data = fn(data)
        if isinstance(data, dict):
            return data["input_ids"], data["labels"]
        i, t = data
        if isinstance(i, (tuple, list)):
            i = i[0]
        if isinstance(t, (tuple, list)):
            t = t[0]
        return i, t

    def _allreduce_dp_grads(self, bucket_bytes: int = 128 << 20):
        """Average stage gradients over the data-parallel group in coalesced
        buckets (one flat copy per bucket; ``FlatDDP`` avoids even that)."""
        from torch._utils import _flatten_dense_tensors, _unflatten_dense_tensors

        n = dist.get_world_size(self.dp_group)
        # DTensor (tensor-parallel) parameters: their local gradient shards
        grads = [p.grad.to_local() if hasattr(p.grad, "to_local") else p.grad
                 for p in self.parameters() if p.grad is not None]
        bucket, size = [], 0
        for g in grads + [None]:
            if g is not None:
                bucket.append(g)
                size += g.numel() * g.element_size()
            if bucket and (g is None or size >= bucket_bytes):
                flat = _flatten_dense_tensors(bucket)
                dist.all_reduce(flat, group=self.dp_group)
                flat.div_(n)
                for t, r in zip(bucket, _unflatten_dense_tensors(flat, bucket)):
                    t.copy_(r)
                bucket, size = [], 0

    def forward(self, ids, targets=None):  # convenience for pp == 1 evaluation
        if len(self.chunks) != 1 or not (self.chunks[0].is_first and self.chunks[0].is_last):
            raise RuntimeError("use train_step() on a multi-stage pipeline")
        return self.chunks[0](ids, targets=targets)


__all__ = ["partition_layers", "PipelineStage", "GPT2Stage", "LlamaStage", "DecoderParts", "DecoderStackStage",
           "SequentialStage", "split_model", "build_pipeline", "PipelineSchedule", "PipelineModule"]
