"""Automatic tensor x pipeline x data sizing for decoder-only LMs on MI355X.

Given a model (this package's GPT-2 / Llama, or any decoder stack
``parallel.pipeline.DecoderParts`` finds), the world size, the sequence
length and micro-batch, this planner enumerates every (tensor t, pipeline p,
data d) with t * p * d = world, t within one node (TP traffic stays on
xGMI), p dividing into the layer count, and scores each with an analytic
model of ONE training step on MI355X:

* memory per GPU: the stage's parameters / t with bf16 weights + grads and
  fp32 master + Adam moments (16 B / parameter), plus the activations the
  1F1B schedule keeps in flight (p micro-batches on the first stage);
  feasible when it fits in ``hbm_gb`` minus a reserve (flash-checkpoint
  staging, allocator slack);
* compute: 6 * params * tokens / (world * peak * efficiency) (8 with
  activation checkpointing);
* TP: 4 all-reduces of [tokens, hidden] bf16 per layer per micro-batch
  (2 forward, 2 backward) at the in-node RCCL bus bandwidth over xGMI;
* PP: the 1F1B bubble (p - 1) / (m + p - 1) of the compute plus the
  boundary transfers;
* DP: the bucketed gradient all-reduce of the stage's parameters (half of
  it hidden under the backward), over xGMI inside a node or the NIC across
  nodes.

Candidates are returned best first; ``auto_accelerate`` takes the first
feasible one for ``("mixed_parallel", "auto")`` (or when not even FSDP fits),
and the dry-run search (``auto_search.py``) can time the top ones.

Parity: ATorch ``auto/opt_lib/shard_planners/dim_planner.py`` (enumerates
tensor x pipe sizes, TeraPipe partition under a memory bound, picks the
cheapest) and ``mip_tp_planner.py`` -- re-designed as a closed-form cost
model of MI355X's HBM, MFMA rate and xGMI links instead of a traced-graph
MIP.
"""

from dataclasses import asdict, dataclass, field
from typing import Dict, List, Optional

import torch.nn as nn

GB = 1e9
GiB = 1 << 30


@dataclass
class Hardware:
    hbm_gb: float = 288.0
    gpus_per_node: int = 8
    bf16_tflops: float = 2500.0  # dense peak per GPU
    efficiency: float = 0.40  # achieved fraction on the GEMMs of a step
    xgmi_link_gbs: float = 153.0  # one link, one direction (a pipeline neighbour exchange)
    # RCCL collectives inside a node spread over the 7 links of each GPU
    # (several rings / channels): bus bandwidth of an in-node all-reduce
    xgmi_busbw_gbs: float = 300.0
    nic_gbs: float = 50.0  # per GPU, across nodes (400 Gb/s)
    reserve_gb: float = 24.0  # staging buffers / allocator slack
    coll_latency_us: float = 20.0  # fixed cost of one RCCL call (launch + sync)


@dataclass
class ModelShape:
    layers: int
    hidden: int
    intermediate: int
    heads: int
    kv_heads: int
    vocab: int
    params: int

    @property
    def layer_params(self) -> float:
        return (self.params - 2 * self.vocab * self.hidden) / max(1, self.layers)


@dataclass
class Plan:
    tensor: int
    pipeline: int
    data: int
    chunks: int
    mem_gb: float
    step_s: float
    feasible: bool
    parts: Dict[str, float] = field(default_factory=dict)

    def as_strategy_cfg(self) -> dict:
        return {"tensor": self.tensor, "pipeline": self.pipeline, "data": self.data, "chunks": self.chunks}

    def as_dict(self) -> dict:
        return asdict(self)


def model_shape(model: nn.Module) -> ModelShape:
    """Layer count / widths of a decoder-only LM."""
    n = sum(p.numel() for p in model.parameters())
    cfg = getattr(model, "cfg", None) or getattr(model, "config", None)

    def g(*names, default=None):
        for k in names:
            v = getattr(cfg, k, None)
            if v is not None:
                return int(v)
        return default

    if cfg is not None and g("num_hidden_layers", "n_layer") is not None:
        hidden = g("hidden_size", "n_embd")
        heads = g("num_attention_heads", "n_head")
        return ModelShape(layers=g("num_hidden_layers", "n_layer"), hidden=hidden,
                          intermediate=g("intermediate_size", "n_inner", default=4 * hidden) or 4 * hidden,
                          heads=heads, kv_heads=g("num_key_value_heads", default=heads) or heads,
                          vocab=g("vocab_size"), params=n)
    from ..parallel.pipeline import DecoderParts

    parts = DecoderParts(model)
    return ModelShape(layers=len(parts.layers), hidden=parts.hidden, intermediate=4 * parts.hidden,
                      heads=max(1, parts.hidden // 128), kv_heads=max(1, parts.hidden // 128), vocab=parts.vocab,
                      params=n)


def _ring_allreduce_s(nbytes: float, n: int, bw_gbs: float) -> float:
    return 0.0 if n <= 1 else 2.0 * (n - 1) / n * nbytes / (bw_gbs * GB)


def estimate(shape: ModelShape, t: int, p: int, d: int, seq: int, micro_batch: int, global_batch: int,
             hw: Hardware, act_ckpt: bool = False) -> Plan:
    world = t * p * d
    m = max(1, global_batch // max(1, d * micro_batch))  # micro-batches per step per pipeline
    tokens_mb = seq * micro_batch
    L, H = shape.layers, shape.hidden
    # parameters of the heaviest stage (the first holds the embedding, the last the head)
    stage_params = (shape.layer_params * (L / p) + shape.vocab * H * (2 if p == 1 else 1)) / t
    state = stage_params * 16
    # activations per layer per micro-batch (bf16 bytes per token): 10 H + 24 H / t (Megatron's
    # 34 H + 5 a s with TP sharding the attention / MLP intermediates; the flash kernel recomputes
    # the scores, so no 5 a s term)
    per_layer = tokens_mb * H * (10 + 24 / t) if not act_ckpt else tokens_mb * H * 2
    in_flight = min(p, m)
    acts = per_layer * (L / p) * in_flight
    logits = tokens_mb * shape.vocab * 4 / t  # fp32 logits of one micro-batch on the last stage
    mem = (state + acts + logits) / GB
    feasible = mem <= hw.hbm_gb - hw.reserve_gb and L % p == 0 and shape.heads % t == 0 and t <= hw.gpus_per_node
    flops = (8 if act_ckpt else 6) * shape.params * seq * global_batch
    compute = flops / (world * hw.bf16_tflops * 1e12 * hw.efficiency)
    # TP: 4 all-reduces per layer per micro-batch on xGMI (ring over t GPUs)
    lat = hw.coll_latency_us * 1e-6
    tp = (_ring_allreduce_s(tokens_mb * H * 2, t, hw.xgmi_busbw_gbs) + lat) * 4 * (L / p) * m if t > 1 else 0.0
    bubble = compute * (p - 1) / (m + p - 1) if p > 1 else 0.0
    # PP boundary: activation + gradient per micro-batch; one neighbour link (xGMI in-node, NIC across)
    pp_bw = hw.xgmi_link_gbs if t * p <= hw.gpus_per_node else hw.nic_gbs
    pp = 2 * m * (tokens_mb * H * 2 / (pp_bw * GB) + lat) if p > 1 else 0.0
    # DP: gradient all-reduce of the stage's parameters (bf16), half hidden under the backward
    dp_bw = hw.xgmi_busbw_gbs if world <= hw.gpus_per_node else hw.nic_gbs
    buckets = max(1.0, stage_params * 2 / (256 << 20))
    dp = 0.5 * _ring_allreduce_s(stage_params * 2, d, dp_bw) + (buckets * lat if d > 1 else 0.0)
    step = compute + tp + bubble + pp + dp
    return Plan(tensor=t, pipeline=p, data=d, chunks=m, mem_gb=round(mem, 2), step_s=step, feasible=feasible,
                parts={"compute": compute, "tp": tp, "bubble": bubble, "pp": pp, "dp": dp,
                       "state_gb": state / GB, "acts_gb": acts / GB})


def plan_3d(model: nn.Module, world: int, seq: int = 4096, micro_batch: int = 1, global_batch: Optional[int] = None,
            hw: Optional[Hardware] = None, act_ckpt: bool = False, shape: Optional[ModelShape] = None) -> List[Plan]:
    """Every (tensor, pipeline, data) factorisation of ``world``, best
    (feasible, then fastest) first."""
    hw = hw or Hardware()
    shape = shape or model_shape(model)
    global_batch = global_batch or max(world, 8) * micro_batch
    out = []
    for t in (1, 2, 4, 8):
        if world % t or t > hw.gpus_per_node:
            continue
        for p in range(1, world // t + 1):
            if (world // t) % p:
                continue
            d = world // (t * p)
            if global_batch % (d * micro_batch):
                continue
            out.append(estimate(shape, t, p, d, seq, micro_batch, global_batch, hw, act_ckpt))
    out.sort(key=lambda x: (not x.feasible, x.step_s))
    return out
