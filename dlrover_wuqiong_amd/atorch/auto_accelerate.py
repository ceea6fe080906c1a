"""``auto_accelerate``: turn a single-device model + optimizer recipe into a
distributed, mixed-precision, memory-optimised training setup.

    status, result, strategy = auto_accelerate(
        model, torch.optim.AdamW, dataset=ds, loss_func=loss_fn,
        optim_args={"lr": 1e-4}, dataloader_args={"batch_size": 64},
        load_strategy=["parallel_mode", ("amp_native", {"dtype": torch.bfloat16}),
                       ("fsdp", {"wrap_cls": (LlamaDecoderLayer,)}), "checkpoint"])
    for batch in result.dataloader:
        out = result.model(**result.prepare_input(batch, device))
        loss = result.loss_func(batch, out)
        loss.backward(); result.optim.step(); result.optim.zero_grad()

Optimizations (applied in a fixed, dependency-respecting order):
  parallel_mode      named groups ``[("data", n)]`` or mixed ``[("tensor", t),
                     ("sequence", s), ("data", d)]`` (``atorch/distributed.py``)
  module_replace     nn.LayerNorm / RMSNorm -> fused HIP norms; transformers models'
                     attention -> the MFMA flash-attention kernels (``hf_attention.py``)
  half               parameters in bf16 (fused optimizers keep fp32 masters)
  amp_native         autocast (bf16 default on MI355X; fp16 adds a GradScaler)
  tensor_parallel    DTensor TP plan inferred from Llama/GPT-style layer names
                     (q/k/v/gate/up column-wise, o/down row-wise)
  checkpoint         activation checkpointing of the given (or decoder) layers
  pipeline_parallel  split GPT2/Llama at decoder layers over the ``("pipeline", p)``
                     dimension; {"chunks": micro-batches, "schedule": "1f1b" |
                     "gpipe" | "interleaved", "virtual_stages": v}; train with
                     ``result.model.train_step(ids, targets)`` (``parallel/pipeline.py``)
  fsdp / zero2       FSDP2 ``fully_shard`` per layer (zero2: no reshard after fwd)
  flat_fsdp /        flat-unit FSDP (``parallel/flat_fsdp.py``): one flat buffer
  flat_zero2         per layer, collectives in place (no copy-in / copy-out),
                     the fused optimizer over the rank's shard; flash
                     checkpoints in ATorch's flat-shard format
  zero1              ZeroRedundancyOptimizer on top of DDP
  ddp                DistributedDataParallel (default when data parallel > 1)

``load_strategy="search"`` (with ``model_fn=`` and ``sample_batch=``) dry-runs
candidate strategies and keeps the fastest (``atorch/auto_search.py``).
``load_strategy="engine"`` runs the acceleration-engine service
(``atorch/engine/``): rank 0 serves a planner/executor, every rank runs the
analyse / tune / dry-run tasks it hands out, and the fastest strategy wins.
``load_strategy=None`` plans semi-automatically from the model size and the
GPU memory (288 GB per MI355X): DDP when weights + grads + Adam states fit in
~70 % of HBM, otherwise FSDP; bf16 autocast always.  (The reference searches
strategies with dry runs + Bayesian optimisation; a deterministic planner
is used here -- no dry-run cost, reproducible choices.)

Parity: ATorch ``atorch/auto/accelerate.py:406`` (``auto_accelerate``) and
``auto/opt_lib/*`` (amp, half, module_replace, checkpoint, zero, fsdp,
parallel_mode, tensor_parallel, sequence_parallel optimizations).
"""

import contextlib
import functools
import os
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.distributed as dist
import torch.nn as nn

from ..common.log import logger
from . import distributed as adist

ORDER = ["parallel_mode", "module_replace", "half", "amp_native", "fp8", "tensor_parallel", "sequence_parallel",
         "context_parallel",
         "checkpoint", "mixed_parallel", "pipeline_parallel", "fsdp", "zero2", "flat_fsdp", "flat_zero2", "zero1",
         "ddp"]
ALIASES = {"amp": "amp_native", "amp_native_bf16": "amp_native", "fsdp2": "fsdp", "zero3": "fsdp",
           "pipe": "pipeline_parallel", "pipeline": "pipeline_parallel", "ds_3d_parallel": "mixed_parallel",
           "deepspeed_3d_parallel": "mixed_parallel", "3d_parallel": "mixed_parallel"}


@dataclass
class Strategy:
    opts: List[Tuple[str, Any]] = field(default_factory=list)

    def names(self) -> List[str]:
        return [n for n, _ in self.opts]

    def config(self, name: str, default=None):
        for n, c in self.opts:
            if n == name:
                return c if c is not None else default
        return default

    @classmethod
    def from_spec(cls, spec) -> "Strategy":
        if isinstance(spec, Strategy):
            return spec
        opts = []
        for item in spec or []:
            name, cfg = (item, None) if isinstance(item, str) else (item[0], item[1] if len(item) > 1 else None)
            opts.append((ALIASES.get(name, name), cfg))
        unknown = [n for n, _ in opts if n not in ORDER]
        if unknown:
            raise ValueError(f"unknown optimizations {unknown}; supported: {ORDER}")
        opts.sort(key=lambda o: ORDER.index(o[0]))
        return cls(opts)


@dataclass
class AutoAccelerateResult:
    model: nn.Module
    optim: Optional[torch.optim.Optimizer] = None
    dataloader: Optional[torch.utils.data.DataLoader] = None
    loss_func: Optional[Callable] = None
    prepare_input: Optional[Callable] = None
    args: Dict[str, Any] = field(default_factory=dict)
    lr_scheduler: Any = None


def _device() -> torch.device:
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _meta_model(model) -> bool:
    from .meta_init import is_meta

    return is_meta(model)


def _default_prepare_input(data, device):
    if torch.is_tensor(data):
        return data.to(device, non_blocking=True)
    if isinstance(data, dict):
        return {k: _default_prepare_input(v, device) for k, v in data.items()}
    if isinstance(data, (list, tuple)):
        return type(data)(_default_prepare_input(v, device) for v in data)
    return data


def _decoder_layer_classes(model: nn.Module) -> Tuple[type, ...]:
    """Repeated transformer blocks: classes of the children of the largest
    ModuleList."""
    best = None
    for m in model.modules():
        if isinstance(m, nn.ModuleList) and len(m) > 1 and (best is None or len(m) > len(best)):
            best = m
    return (type(best[0]),) if best is not None else ()


def plan_strategy(model: nn.Module, world: int, gpu_mem_gb: float = 288.0) -> Strategy:
    n = sum(p.numel() for p in model.parameters())
    # bf16 weights + fp32 grads accumulation buffer + fp32 master + 2 Adam moments
    need_gb = n * (2 + 4 + 4 + 8) / 2 ** 30
    opts: List[Tuple[str, Any]] = [("parallel_mode", None), ("module_replace", None),
                                   ("amp_native", {"dtype": torch.bfloat16})]
    if world > 1:
        opts.append(("fsdp", None) if need_gb > 0.7 * gpu_mem_gb else ("ddp", None))
    elif need_gb > 0.7 * gpu_mem_gb:
        opts.append(("checkpoint", None))
    logger.info(f"auto_accelerate plan for {n / 1e9:.2f}B params ({need_gb:.1f} GB of training state) "
                f"on {world} rank(s): {[o[0] for o in opts]}")
    return Strategy.from_spec(opts)


# ------------------------------------------------------------ optimizations
def _apply_parallel_mode(ctx, cfg):
    if not dist.is_initialized():
        if int(os.getenv("WORLD_SIZE", "1")) > 1:
            adist.init_distributed("nccl")
        else:
            return
    world = dist.get_world_size()
    config = cfg or ([("data", world)], None)
    if adist.parallel_config() is None:
        adist.create_parallel_group(config)
    ctx["dp_group"] = adist.parallel_group("data")
    ctx["zero_group"] = adist.parallel_group("zero")
    ctx["tp_group"] = adist.parallel_group("tensor")
    ctx["sp_group"] = adist.parallel_group("sequence")


def _replace_norms(model: nn.Module):
    from ..ops.norm import LayerNorm, RMSNorm

    n = 0
    for name, mod in list(model.named_modules()):
        for cname, child in list(mod.named_children()):
            if type(child) is nn.LayerNorm and child.elementwise_affine and len(child.normalized_shape) == 1:
                new = LayerNorm(child.normalized_shape[0], eps=child.eps, bias=child.bias is not None,
                                device=child.weight.device, dtype=child.weight.dtype)
                new.load_state_dict(child.state_dict())
                setattr(mod, cname, new)
                n += 1
            elif type(child).__name__ in ("LlamaRMSNorm", "RMSNorm") and not isinstance(child, RMSNorm) \
                    and hasattr(child, "weight"):
                eps = getattr(child, "variance_epsilon", getattr(child, "eps", 1e-6))
                new = RMSNorm(child.weight.shape[0], eps=eps, device=child.weight.device, dtype=child.weight.dtype)
                with torch.no_grad():
                    new.weight.copy_(child.weight)
                setattr(mod, cname, new)
                n += 1
    return n


def _replace_linears(model: nn.Module) -> int:
    """Plain ``nn.Linear`` -> ``ops.linear.FusedLinear`` (same module, class
    swapped): once a flat buffer owns the weight (FlatParams / FlatFSDP set
    ``_dwamd_direct``) the weight gradient GEMM accumulates straight into the
    flat gradient on a side stream; otherwise it is ``F.linear`` as before.
    Without it autograd zero-fills and then adds every weight gradient (two
    extra passes per projection: 10 ms per Llama-3-8B step)."""
    from ..ops.linear import FusedLinear

    n = 0
    for m in model.modules():
        if type(m) is nn.Linear:
            m.__class__ = FusedLinear
            n += 1
    return n


def _apply_module_replace(ctx, cfg):
    from .hf_attention import enable_dwamd_attention

    n = _replace_norms(ctx["model"])
    nl = _replace_linears(ctx["model"])
    hf = enable_dwamd_attention(ctx["model"])
    logger.info(f"module_replace: {n} norm layers -> fused HIP norms, {nl} Linear -> FusedLinear"
                + ("; HF attention -> MFMA flash attention" if hf else ""))


def _apply_half(ctx, cfg):
    # ("half", "fp16" | "bf16") as in the reference, or {"dtype": ...}
    if isinstance(cfg, str):
        dtype = torch.float16 if cfg.lower() in ("fp16", "float16", "half") else torch.bfloat16
    else:
        dtype = (cfg or {}).get("dtype", torch.bfloat16) if isinstance(cfg, dict) else torch.bfloat16
    ctx["model"].to(dtype)


class _AutocastModule(nn.Module):
    def __init__(self, module: nn.Module, dtype):
        super().__init__()
        self.module = module
        self.dtype = dtype

    def forward(self, *a, **kw):
        dev = "cuda" if torch.cuda.is_available() else "cpu"
        with torch.autocast(dev, dtype=self.dtype):
            return self.module(*a, **kw)


def _autocast_fn(fn, dtype):
    @functools.wraps(fn)
    def run(*a, **kw):
        with torch.autocast("cuda" if torch.cuda.is_available() else "cpu", dtype=dtype):
            return fn(*a, **kw)

    return run


def _apply_amp_native(ctx, cfg):
    dtype = (cfg or {}).get("dtype", torch.bfloat16) if isinstance(cfg, dict) else torch.bfloat16
    ctx["amp_dtype"] = dtype
    if dtype == torch.float16:
        ctx["grad_scaler"] = torch.amp.GradScaler("cuda" if torch.cuda.is_available() else "cpu")


def _apply_fp8(ctx, cfg):
    """ATorch ``fp8`` (amp_optimization.py Fp8Optimization): eligible
    ``nn.Linear`` layers -> ``ops.fp8.Fp8Linear`` (FP8 GEMMs on the CDNA4
    matrix cores, delayed scaling advanced after every optimizer step)."""
    from ..ops import fp8

    cfg = cfg if isinstance(cfg, dict) else {}
    if ctx.get("tp_like"):
        # the TP layers replace the Linears fp8 would have converted: refuse
        # loudly instead of silently training in bf16
        raise ValueError("fp8 cannot be combined with tensor / sequence / mixed parallelism: drop 'fp8' from the "
                         "strategy, or use it with DDP / FSDP")
    fp8.configure(history_len=int(cfg.get("amax_history_len", 1024)), margin=int(cfg.get("margin", 0)),
                  algo=cfg.get("amax_compute_algo", "max"), reduce_amax=bool(cfg.get("reduce_amax", True)),
                  interval=int(cfg.get("interval", 1)), group=ctx.get("dp_group"))
    done = fp8.replace_linears(ctx["model"], include=cfg.get("include"), exclude=cfg.get("exclude"),
                               fp8_format=cfg.get("fp8_format", "HYBRID"))
    ctx["fp8"] = done
    logger.info(f"fp8: {len(done)} nn.Linear -> Fp8Linear ({cfg.get('fp8_format', 'HYBRID')})")


def _tp_plan_for(model: nn.Module):
    from torch.distributed.tensor.parallel import ColwiseParallel, RowwiseParallel

    col = ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "c_fc", "fc1", "w1", "w3", "query_key_value",
           "query", "key", "value", "dense_h_to_4h")
    row = ("o_proj", "down_proj", "c_proj", "fc2", "w2", "dense", "out_proj", "dense_4h_to_h")
    # encoder families (Bert / RoBERTa / ViT): the MLP's first Linear is
    # ``intermediate.dense`` -- column, although plain ``dense`` is a row one
    col2 = ("intermediate.dense",)
    plan = {}
    for name, m in model.named_modules():
        if not isinstance(m, nn.Linear):
            continue
        leaf = name.rsplit(".", 1)[-1]
        last2 = ".".join(name.rsplit(".", 2)[-2:])
        if last2 in col2 or leaf in col:
            plan[name] = ColwiseParallel()
        elif leaf in row:
            plan[name] = RowwiseParallel()
    return plan


def _fix_attention_heads(model: nn.Module, tp: int):
    """HF attention modules keep their head counts as attributes: divide them
    so views match the local shards."""
    for m in model.modules():
        for attr in ("num_heads", "num_key_value_heads", "num_attention_heads", "n_head"):
            v = getattr(m, attr, None)
            if isinstance(v, int) and v % tp == 0 and not isinstance(m, nn.Linear):
                setattr(m, attr, v // tp)
        if hasattr(m, "hidden_size") and isinstance(getattr(m, "hidden_size"), int) and hasattr(m, "num_heads"):
            m.hidden_size = m.hidden_size // tp
        # Bert-style self-attention: the merged-heads width of the context
        if isinstance(getattr(m, "all_head_size", None), int) and hasattr(m, "num_attention_heads"):
            m.all_head_size = m.all_head_size // tp


def _dtensor_tp(model, mesh, tp: int, cfg=None) -> int:
    """Shard ``model``'s Megatron blocks over ``mesh`` with DTensor
    (colwise -> rowwise: one all-reduce per block each way); returns the
    number of Linear layers sharded."""
    from torch.distributed.tensor.parallel import parallelize_module

    plan = (cfg or {}).get("plan") if isinstance(cfg, dict) else None
    heads = {}
    if plan is None and not (isinstance(cfg, dict) and cfg.get("planner") == "names"):
        # structural plan (torch.fx): Megatron column -> row blocks whatever
        # the layers are called; the name table only as a fallback
        from .tp_planner import auto_tp_plan

        plan = auto_tp_plan(model, heads) or None
    plan = plan or _tp_plan_for(model)
    parallelize_module(model, mesh, plan)
    if heads:
        from .tp_planner import shrink_head_attributes

        shrink_head_attributes(model, heads, tp)
    _fix_attention_heads(model, tp)
    return len(plan)


def _megatron_tp(model, group, tp: int, cfg=None) -> int:
    """Swap ``model``'s Megatron blocks (found structurally by the fx
    planner, else by layer names) for this package's Column / Row parallel
    Linears over ``group``: blocking autograd collectives on the tensor
    group (RCCL over xGMI), deterministic on gloo too.  Returns the number
    of Linear layers swapped."""
    from torch.distributed.tensor.parallel import ColwiseParallel

    from ..parallel.tensor_parallel import ColumnParallelLinear, RowParallelLinear

    plan = (cfg or {}).get("plan") if isinstance(cfg, dict) else None
    heads = {}
    if plan is None:
        from .tp_planner import auto_tp_plan

        plan = dict(auto_tp_plan(model, heads) or {})
        # blocks the tracer could not prove (e.g. HF attention with control
        # flow): the name table's remaining entries, taken per layer when
        # they hold both a column and a row Linear -- grouped per layer (the path up to the first list index), so an
        # attention block split over sibling modules (Bert: attention.self.
        # query/key/value -> attention.output.dense) is taken as a whole
        def layer_of(name):
            parts = name.split(".")
            for k, x in enumerate(parts):
                if x.isdigit():
                    return ".".join(parts[:k + 1])
            return name.rsplit(".", 1)[0] if "." in name else ""

        by_layer = {}
        for name, style in _tp_plan_for(model).items():
            if name not in plan:
                by_layer.setdefault(layer_of(name), {})[name] = style
        for entries in by_layer.values():
            kinds = {isinstance(v, ColwiseParallel) for v in entries.values()}
            if kinds == {True, False}:
                plan.update(entries)
    plan = plan or _tp_plan_for(model)
    for name, style in plan.items():
        lin = model.get_submodule(name)
        parent = model.get_submodule(name.rsplit(".", 1)[0]) if "." in name else model
        col = isinstance(style, ColwiseParallel) or style == "colwise"
        new = (ColumnParallelLinear if col else RowParallelLinear).from_linear(lin, group)
        setattr(parent, name.rsplit(".", 1)[-1], new)
    if heads:
        from .tp_planner import shrink_head_attributes

        shrink_head_attributes(model, heads, tp)
    _fix_attention_heads(model, tp)
    return len(plan)


def _apply_tensor_parallel(ctx, cfg):
    from torch.distributed.device_mesh import DeviceMesh

    _g, ranks = adist.parallel_group_and_ranks("tensor")
    if not ranks or len(ranks) == 1:
        return
    mesh = DeviceMesh("cuda" if torch.cuda.is_available() else "cpu", ranks, mesh_dim_names=("tensor",))
    n = _dtensor_tp(ctx["model"], mesh, len(ranks), cfg)
    ctx["tp_mesh"] = mesh
    logger.info(f"tensor_parallel: {n} linear layers sharded over {len(ranks)} ranks")


def _apply_sequence_parallel(ctx, cfg):
    """Ulysses sequence parallel (ATorch ``SequenceParallelOptimization``):
    ``{"sp_size": n, "module": cls | (cls, ...) | None, "set_sp_func_name":
    "set_sp", "batch_sp_processing_fn": fn(batch, sp_size, sp_rank)}``.
    Creates the SP groups (consecutive ranks: one xGMI-connected node), calls
    ``set_sp(sp_size, sp_rank, sp_group)`` on the model (or on every module of
    the given classes) and splits each batch along the sequence in
    ``prepare_input``; the ranks of one SP group read the same batch."""
    cfg = cfg if isinstance(cfg, dict) else {"sp_size": cfg or 0}
    size = int(cfg.get("sp_size", cfg.get("size", 0)) or 0)
    if size <= 1:
        return
    if adist.get_sequence_parallel_group() is None:
        adist.create_sequence_parallel_group(size)
    group, rank = adist.get_sequence_parallel_group(), adist.get_sequence_parallel_rank()
    fname = cfg.get("set_sp_func_name", "set_sp")
    mods = cfg.get("module")
    model = ctx["model"]
    if mods is None:
        targets = [model] if hasattr(model, fname) else []
    else:
        mods = tuple(mods) if isinstance(mods, (list, tuple)) else (mods,)
        targets = [m for m in model.modules() if isinstance(m, mods)]
    for m in targets:
        getattr(m, fname)(size, rank, group)
    if not targets:
        logger.warning(f"sequence_parallel: no module with {fname}(); only the SP groups were created")
    ctx["sp"] = (size, rank, cfg.get("batch_sp_processing_fn"))
    logger.info(f"sequence_parallel: {size}-way, {len(targets)} {fname}() call(s)")


def _apply_context_parallel(ctx, cfg):
    """Context parallel (``parallel/context_parallel.py``): ``{"cp_size": n,
    "set_cp_func_name": "set_cp"}`` or just ``n``.  Uses the sequence
    parallel groups (consecutive ranks of one node), calls ``set_cp(group)``
    on the model and, in ``prepare_input``, takes this rank's zig-zag shard
    of every [batch, seq, ...] tensor of the batch; the CP ranks of a group
    read the same batch and their gradients average like data parallel."""
    cfg = cfg if isinstance(cfg, dict) else {"cp_size": cfg or 0}
    size = int(cfg.get("cp_size", cfg.get("size", 0)) or 0)
    if size <= 1:
        return
    if ctx.get("sp"):
        raise ValueError("context_parallel and sequence_parallel share the sequence groups; use one of them")
    if adist.get_sequence_parallel_group() is None:
        adist.create_sequence_parallel_group(size)
    group, rank = adist.get_sequence_parallel_group(), adist.get_sequence_parallel_rank()
    fname = cfg.get("set_cp_func_name", "set_cp")
    targets = [m for m in ctx["model"].modules() if hasattr(m, fname)][:1]
    if not targets:
        raise ValueError(f"context_parallel: the model has no {fname}() method")
    getattr(targets[0], fname)(group)

    def split(batch, _size, _rank):
        from ..parallel.context_parallel import zigzag_split

        def one(t):
            return zigzag_split(t, group, dim=1) if torch.is_tensor(t) and t.dim() >= 2 else t

        if isinstance(batch, dict):
            return {k: one(v) for k, v in batch.items()}
        if isinstance(batch, (list, tuple)):
            return type(batch)(one(v) for v in batch)
        return one(batch)

    ctx["sp"] = (size, rank, cfg.get("batch_cp_processing_fn") or split)
    logger.info(f"context_parallel: {size}-way (zig-zag shards, K/V all-gather)")


def _wrap_cls(ctx, cfg):
    cls = None
    if isinstance(cfg, dict):
        cls = cfg.get("wrap_cls") or cfg.get("wrap_class") or cfg.get("atorch_wrap_cls")
    elif isinstance(cfg, (list, tuple)):
        cls = cfg
    if cls is None:
        cls = _decoder_layer_classes(ctx["model"])
    return tuple(cls) if isinstance(cls, (list, tuple)) else (cls,)


def _apply_checkpoint(ctx, cfg):
    from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import apply_activation_checkpointing

    import functools as _ft

    from torch.distributed.algorithms._checkpoint.checkpoint_wrapper import checkpoint_wrapper

    from ..parallel.randomizer import rng_checkpoint

    classes = _wrap_cls(ctx, cfg)
    if classes:
        # the recompute also replays the parallel randomizer / tracked RNG
        # states (dropout inside a forked stream regenerates its mask)
        apply_activation_checkpointing(ctx["model"], check_fn=lambda m: isinstance(m, classes),
                                       checkpoint_wrapper_fn=_ft.partial(checkpoint_wrapper,
                                                                         checkpoint_fn=rng_checkpoint))
        logger.info(f"checkpoint: activation checkpointing on {[c.__name__ for c in classes]}")


def _apply_pipeline_parallel(ctx, cfg):
    from ..parallel.pipeline import PipelineModule

    cfg = cfg if isinstance(cfg, dict) else {}
    group, ranks = adist.parallel_group_and_ranks("pipeline")
    if not ranks or len(ranks) == 1:
        return
    me = dist.get_rank()
    emb_group = None
    # first + last stage of every pipeline group (created by every rank, same order)
    for _g, rk in adist.parallel_groups_and_ranks_all("pipeline"):
        eg = dist.new_group(sorted({rk[0], rk[-1]}))
        if me in rk:
            emb_group = eg
    pipe = PipelineModule(ctx["model"], len(ranks), ranks.index(me),
                          num_microbatches=cfg.get("chunks", cfg.get("num_microbatches", len(ranks))),
                          schedule=cfg.get("schedule", "1f1b"), virtual_stages=cfg.get("virtual_stages", 1),
                          group=group, embedding_group=emb_group)
    pipe.amp_dtype = ctx.get("amp_dtype")
    ctx["model"] = pipe
    ctx["pipeline"] = True
    logger.info(f"pipeline_parallel: stage {pipe.stage}/{len(ranks)} "
                f"layers {[(c.start, c.end) for c in pipe.chunks]} schedule {pipe.schedule_name}")


def _mixed_cfg(cfg) -> Dict[str, Any]:
    """mixed_parallel config as a dict: a dict, or a config object such as
    the reference's ``DeepSpeed3DParallelConfig`` (its ``ds_config`` -- dict
    or JSON path -- supplies ``gradient_accumulation_steps`` as the
    micro-batch count)."""
    if cfg is None:
        return {}
    if isinstance(cfg, str):
        return {"auto": True} if cfg == "auto" else {}
    out = dict(cfg) if isinstance(cfg, dict) else {k: v for k, v in vars(cfg).items() if not k.startswith("_")}
    ds = out.get("ds_config")
    if isinstance(ds, str) and os.path.exists(ds):
        import json

        with open(ds) as f:
            ds = json.load(f)
    if isinstance(ds, dict) and "chunks" not in out and ds.get("gradient_accumulation_steps"):
        out["chunks"] = int(ds["gradient_accumulation_steps"])
    return out


def _apply_mixed_parallel(ctx, cfg):
    """TP x PP x DP in one strategy (ATorch ``MixedParallelOptimization`` /
    ``ds_3d_parallel``; reference auto/opt_lib/mixed_parallel_optimization.py:32,
    ds_3d_parallel_optimization.py:55): ``{"tensor": t, "pipeline": p,
    "data": d, "chunks": m, "schedule": "1f1b", "virtual_stages": v}``.

    Rank layout tensor -> pipeline -> data (TP inside one node's xGMI mesh,
    PP / DP across).  The unsharded model is rebuilt with the framework's
    Megatron-style TP layers (fused QKV / gate|up regrouped per rank,
    vocab-parallel embedding, LM head and cross-entropy), cut into pipeline
    stages at decoder-layer boundaries, and the stage's gradients average
    over the data group after every pipeline step.  Train with
    ``result.model.train_step(ids, targets)``."""
    from ..models.llama import Llama, shard_llama_state_dict
    from ..parallel.pipeline import PipelineModule

    cfg = _mixed_cfg(cfg)
    if not dist.is_initialized():
        raise RuntimeError("mixed_parallel needs torch.distributed")
    world = dist.get_world_size()
    # sizes from the config, else from the parallel_mode groups
    t = int(cfg.get("tensor") or adist.parallel_group_size("tensor") or 1)
    p = int(cfg.get("pipeline") or adist.parallel_group_size("pipeline") or 1)
    d = int(cfg.get("data") or world // max(1, t * p))
    if t * p * d != world:
        raise ValueError(f"mixed_parallel: tensor {t} x pipeline {p} x data {d} != world {world}")
    if adist.parallel_config() is None:
        adist.create_parallel_group(([("tensor", t), ("pipeline", p), ("data", d)], None))
    model = ctx["model"]
    if t > 1:
        tg, tranks = adist.parallel_group_and_ranks("tensor")
        if isinstance(model, Llama):
            # this package's Llama: Megatron TP layers (fused QKV / gate|up
            # regrouped per rank, vocab-parallel embedding + head + CE)
            tr = adist.parallel_rank("tensor")
            dtype = next(model.parameters()).dtype
            full = {k: v.detach() for k, v in model.state_dict().items()}
            tp_model = Llama(model.cfg, tp_group=tg).to(dtype)
            tp_model.load_state_dict(shard_llama_state_dict(full, model.cfg, tr, t))
            model = tp_model
        else:
            # any other model: the structural (torch.fx) Megatron plan,
            # realised with this package's Column / Row parallel Linears on
            # the existing tensor group (no new communicators)
            n = _megatron_tp(model, tg, t, cfg.get("tp_cfg"))
            if n == 0:
                raise ValueError(f"mixed_parallel: no tensor-parallel block found in {type(model).__name__}")
    if p > 1:
        group, ranks = adist.parallel_group_and_ranks("pipeline")
        me = dist.get_rank()
        emb_group = None
        for _g, rk in adist.parallel_groups_and_ranks_all("pipeline"):
            eg = dist.new_group(sorted({rk[0], rk[-1]}))
            if me in rk:
                emb_group = eg
        split_kw = {k: cfg[k] for k in ("loss_fn", "boundary_shape") if k in cfg}
        model = PipelineModule(model, p, ranks.index(me), num_microbatches=cfg.get("chunks", p),
                               schedule=cfg.get("schedule", "1f1b"), virtual_stages=cfg.get("virtual_stages", 1),
                               group=group, embedding_group=emb_group, **split_kw)
        model.amp_dtype = ctx.get("amp_dtype")
        model.batch_fn = cfg.get("batch_fn")
        ctx["pipeline"] = True
    ctx["model"] = model
    ctx["dp_group"] = adist.parallel_group("data")
    ctx["tp_group"] = adist.parallel_group("tensor")
    logger.info(f"mixed_parallel: tensor {t} x pipeline {p} x data {d}")


def _hsdp_mesh(ctx):
    """Hybrid sharding (HSDP): with ``parallel_mode`` groups ("zero", z) and
    ("data", d), both > 1, parameters are sharded inside each zero group and
    replicated across the data groups -- a 2-D FSDP2 mesh
    (replicate = data, shard = zero): reduce-scatter within a node's xGMI
    group, all-reduce of the shards across nodes.  Parity: ATorch
    zero_optimization.py:377-394 (FSDP HYBRID_SHARD)."""
    zg, dpg = ctx.get("zero_group"), ctx.get("dp_group")
    if zg is None or dpg is None or dist.get_world_size(zg) <= 1 or dist.get_world_size(dpg) <= 1:
        return None
    if dist.get_world_size(zg) * dist.get_world_size(dpg) != dist.get_world_size():
        raise ValueError("HSDP needs zero x data == world size (no other parallel dimensions)")
    from torch.distributed.device_mesh import DeviceMesh

    rows = sorted(sorted(r) for _g, r in adist.parallel_groups_and_ranks_all("zero"))
    data_groups = {tuple(sorted(r)) for _g, r in adist.parallel_groups_and_ranks_all("data")}
    cols = {tuple(sorted(row[j] for row in rows)) for j in range(len(rows[0]))}
    if cols != data_groups:
        raise ValueError(f"zero groups {rows} and data groups {sorted(data_groups)} do not form a 2-D grid")
    mesh = DeviceMesh("cuda" if torch.cuda.is_available() else "cpu", torch.tensor(rows),
                      mesh_dim_names=("replicate", "shard"))
    logger.info(f"fsdp: hybrid sharding over a {len(rows)} x {len(rows[0])} (replicate x shard) mesh")
    return mesh


def _apply_fsdp(ctx, cfg, reshard=True):
    from torch.distributed.fsdp import MixedPrecisionPolicy, fully_shard

    if not dist.is_initialized():
        return
    classes = _wrap_cls(ctx, cfg)
    dtype = ctx.get("amp_dtype")
    mp = MixedPrecisionPolicy(param_dtype=dtype, reduce_dtype=torch.float32) if dtype else MixedPrecisionPolicy()
    mesh = _hsdp_mesh(ctx)
    local_sgd = isinstance(cfg, dict) and cfg.get("use_local_sgd")
    if local_sgd:
        if mesh is None:
            raise RuntimeError("use_local_sgd requires hybrid sharding (parallel_mode zero x data)")
        # every replica is its own FSDP group over the shard dimension: no
        # per-step all-reduce across replicas at all; HSDPLocalSGD merges the
        # shards every sync_interval steps (and averages gradients in warm-up)
        ctx["local_sgd"] = (mesh.get_group("replicate"), cfg)
        mesh = mesh["shard"]
    dpg = ctx.get("dp_group")
    if mesh is None and not local_sgd and dpg is not None and dist.get_world_size(dpg) != dist.get_world_size():
        from torch.distributed.device_mesh import DeviceMesh

        _g, ranks = adist.parallel_group_and_ranks("data")
        mesh = DeviceMesh("cuda" if torch.cuda.is_available() else "cpu", ranks, mesh_dim_names=("data",))
    model = ctx["model"]
    cfgd = dict(cfg) if isinstance(cfg, dict) else {}
    if cfgd.get("optim_in_backward"):
        # each unit's optimizer update from its post-backward reduce-scatter,
        # on a side stream under the rest of the backward (optimizers/in_backward.py)
        ctx["optim_in_backward"] = True
    # meta-device model (init_empty_weights / torch.device("meta")): shard
    # first, then materialise only this rank's shards (atorch/meta_init.py)
    from . import meta_init

    here_meta = meta_init.is_meta(model)
    flags = torch.tensor([int(here_meta), int(not here_meta and dist.get_rank() == 0)], dtype=torch.int64)
    flags_dev = flags.to(_device()) if dist.get_backend() != "gloo" else flags
    dist.all_reduce(flags_dev, op=dist.ReduceOp.MAX)
    any_meta, rank0_real = (bool(x) for x in flags_dev.cpu().tolist())
    sync = bool(cfgd.get("sync_module_states"))
    full_rank0 = None
    if any_meta:
        if here_meta is False and dist.get_rank() != 0:
            raise RuntimeError("meta-device init: a rank other than 0 holds a real model while others are meta")
        if rank0_real and not sync:
            raise ValueError("rank 0 holds a real model and the other ranks a meta one: pass "
                             "sync_module_states=True to scatter rank 0's weights")
        if rank0_real:
            full_rank0 = meta_init.capture_full_states(model) if dist.get_rank() == 0 else None
            cfgd["_rank0_real"] = True
    elif sync:
        # every rank built the full model: rank 0's initial weights win
        meta_init.sync_full_module_states(model, src=0)
        logger.info("fsdp: sync_module_states -- parameters and buffers broadcast from rank 0")
    extra = {}
    if isinstance(cfg, dict) and cfg.get("cpu_offload"):
        # parameters, gradients and optimizer state live on the host; the
        # optimizer step runs there (reference zero_optimization cpu_offload)
        from torch.distributed.fsdp import CPUOffloadPolicy

        extra["offload_policy"] = CPUOffloadPolicy()
    n = 0
    # activation checkpointing runs first: shard the CheckpointWrapper, not
    # the layer inside it.  FSDP(CheckpointWrapper(layer)) casts the layer
    # inputs to param_dtype once, before the checkpointed region; the
    # inverted nesting recomputes on uncast fp32 inputs (FSDP2 skips its
    # input cast in the pre-backward recompute) and the recomputed saved
    # tensors no longer match the forward ones.
    ckpt_inner = {id(m._checkpoint_wrapped_module) for m in model.modules()
                  if getattr(m, "_checkpoint_wrapped_module", None) is not None}
    # bottom-up (children before parents, as fully_shard requires): nested
    # wrap classes, e.g. (DecoderLayer, MLP), each become their own FSDP unit
    for m in reversed(list(model.modules())):
        if not classes or m is model or id(m) in ckpt_inner:
            continue
        inner = getattr(m, "_checkpoint_wrapped_module", None)
        if isinstance(m, classes) or (inner is not None and isinstance(inner, classes)):
            fully_shard(m, mesh=mesh, mp_policy=mp, reshard_after_forward=reshard, **extra)
            n += 1
    fully_shard(model, mesh=mesh, mp_policy=mp, reshard_after_forward=reshard, **extra)
    if any_meta:
        dev = torch.device("cpu") if cfgd.get("cpu_offload") else _device()
        how = meta_init.materialize_sharded(model, dev, cfgd, full_rank0)
        del full_rank0
        logger.info(f"fsdp: meta-device model materialised per shard on {dev} ({how})")
        ctx["meta_init"] = how
    ctx["fsdp"] = True
    ctx.pop("amp_dtype_autocast", None)
    logger.info(f"fsdp: {n} layers sharded (reshard_after_forward={reshard})")


def _apply_flat_fsdp(ctx, cfg, reshard=True):
    """Flat-unit FSDP over the data-parallel group (every rank at world 1):
    the optimizer built below is the fused flat one over the rank's shard."""
    from ..parallel.flat_fsdp import FlatFSDP

    cfgd = dict(cfg) if isinstance(cfg, dict) else {}
    model = ctx["model"]
    meta = _meta_model(model)
    if not meta:
        model = model.to(_device())  # the flat buffers are built where the parameters are
    pg = ctx.get("dp_group") if dist.is_initialized() else None
    rg = None
    zg = ctx.get("zero_group") if dist.is_initialized() else None
    if zg is not None and pg is not None and dist.get_world_size(zg) > 1 and dist.get_world_size(pg) > 1:
        # parallel_mode ("zero", z) x ("data", d): shard within the zero group,
        # replicate across the data groups (hybrid sharding, as fsdp's 2-D mesh)
        pg, rg = zg, pg
    # a meta-device model is materialised per shard (sharding-invariant
    # counter-based init, atorch/meta_init.py); init_seed / buffer_init_fn as for fsdp
    ctx["model"] = FlatFSDP(model, wrap_cls=_wrap_cls(ctx, cfg), process_group=pg,
                            reshard_after_forward=cfgd.get("reshard_after_forward", reshard),
                            sync_module_states=cfgd.get("sync_module_states", True), device=_device(),
                            init_seed=int(cfgd.get("init_seed", 0)), buffer_init_fn=cfgd.get("buffer_init_fn"),
                            replicate_group=rg)
    if meta:
        ctx["meta_init"] = "flat_deterministic"
    ctx["flat_fsdp"] = ctx["model"]
    ctx["fsdp"] = True  # no DDP on top; autocast is the caller's (use "half": bf16 parameters)


def _apply_ddp(ctx, cfg):
    if not dist.is_initialized() or ctx.get("fsdp"):
        return
    dpg = ctx.get("dp_group")
    if ctx.get("pipeline"):
        # the pipeline all-reduces stage gradients over the data dimension
        if dpg is not None and dist.get_world_size(dpg) > 1:
            ctx["model"].dp_group = dpg
        return
    if adist.parallel_config() is not None and dpg is None:
        return  # the parallel config has no data-parallel dimension
    if dpg is not None and dist.get_world_size(dpg) == 1:
        return
    kw = dict(cfg) if isinstance(cfg, dict) else {}
    kw.setdefault("find_unused_parameters", ctx.get("find_unused_parameters", False))
    dev = _device()
    eps = {getattr(m, "ep", 1) for m in ctx["model"].modules() if hasattr(m, "experts") and hasattr(m, "ep")}
    if max(eps, default=1) > 1:
        # expert-parallel MoE: experts differ across an EP group -- their
        # grads go over the expert-data-parallel group, the rest through DDP
        from ..parallel.moe_ddp import MoEDistributedDataParallel, expert_data_parallel_group

        ep = max(eps)
        edp = kw.pop("expert_dp_group", None) or expert_data_parallel_group(ep)
        ctx["model"] = MoEDistributedDataParallel(ctx["model"], expert_dp_group=edp, process_group=dpg,
                                                  device_ids=[dev.index] if dev.type == "cuda" else None, **kw)
        ctx["moe_ddp"] = ctx["model"]
        logger.info(f"ddp: MoE-aware (EP {ep}; expert grads over the expert-data-parallel group)")
        return
    ctx["model"] = nn.parallel.DistributedDataParallel(
        ctx["model"], device_ids=[dev.index] if dev.type == "cuda" else None, process_group=dpg, **kw)


APPLY = {"parallel_mode": _apply_parallel_mode, "module_replace": _apply_module_replace, "half": _apply_half,
         "amp_native": _apply_amp_native, "fp8": _apply_fp8, "tensor_parallel": _apply_tensor_parallel,
         "sequence_parallel": _apply_sequence_parallel, "context_parallel": _apply_context_parallel,
         "checkpoint": _apply_checkpoint, "mixed_parallel": _apply_mixed_parallel,
         "pipeline_parallel": _apply_pipeline_parallel,
         "fsdp": _apply_fsdp, "zero2": functools.partial(_apply_fsdp, reshard=False),
         "flat_fsdp": _apply_flat_fsdp, "flat_zero2": functools.partial(_apply_flat_fsdp, reshard=False),
         "zero1": lambda ctx, cfg: ctx.__setitem__("zero1", True), "ddp": _apply_ddp}


def _flat_optimizer(fs, optim_func, args):
    """The fused flat optimizer over a FlatFSDP shard for torch / ATorch
    AdamW, Adam and AGD (the shard is one flat buffer: per-parameter groups
    do not apply)."""
    from ..optimizers.fused import FusedAdamW, FusedAGD

    name = getattr(optim_func, "__name__", str(optim_func))
    a = dict(args)
    if name in ("AdamW", "FusedAdamW", "MultiTensorAdamW", "Adam"):
        kw = {k: a[k] for k in ("lr", "betas", "eps", "weight_decay") if k in a}
        if "max_grad_norm" in a:
            kw["max_grad_norm"] = a["max_grad_norm"]
        return FusedAdamW(fs.shard_flat, adamw=name != "Adam", **kw)
    if name in ("AGD", "FusedAGD", "MultiTensorAGD"):
        kw = {k: a[k] for k in ("lr", "betas", "delta", "weight_decay") if k in a}
        return FusedAGD(fs.shard_flat, **kw)
    raise ValueError(f"flat_fsdp: no fused flat optimizer for {name} (AdamW / Adam / AGD)")


_PARTITION: List[int] = []  # [rank, size] of the last auto_accelerate's data partition


def _data_partition(ctx) -> Tuple[int, int]:
    """(rank, size) of this process among the replicas that read distinct
    batches: the data-parallel group, with SP groups sharing a batch and
    zero (sharding) ranks each reading their own."""
    init = dist.is_initialized()
    dpg = ctx.get("dp_group")
    dp_size = dist.get_world_size(dpg) if (init and dpg is not None) else (dist.get_world_size() if init else 1)
    dp_rank = dist.get_rank(dpg) if (init and dpg is not None) else (dist.get_rank() if init else 0)
    if ctx.get("sp") and init and dp_size == dist.get_world_size():
        # the data group spans the SP groups (ATorch: SP is independent of
        # DP): the ranks of one SP group share a batch -> one sampler
        # replica per group (gradients still average over every rank)
        sp = ctx["sp"][0]
        dp_size, dp_rank = dp_size // sp, dp_rank // sp
    zg = ctx.get("zero_group")
    if zg is not None and dist.get_world_size(zg) > 1:
        # zero (sharding) ranks are data parallel too: each reads its own batch
        dp_rank = dp_rank * dist.get_world_size(zg) + dist.get_rank(zg)
        dp_size = dp_size * dist.get_world_size(zg)
    return dp_rank, dp_size


def get_data_partition_rank_and_size() -> Tuple[int, int]:
    """Data-partition (rank, size) chosen by the last ``auto_accelerate`` call
    -- what a user-built DataLoader's sampler needs (reference:
    atorch/atorch/auto/model_context.py ``get_data_partition_rank_and_size``).
    Before any call: the global rank / world size."""
    if _PARTITION:
        return _PARTITION[0], _PARTITION[1]
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def auto_accelerate(model: nn.Module, optim_func=None, dataset=None, loss_func=None, prepare_input=None,
                    model_input_format=None, optim_args=None, optim_param_func=None, dataloader_args=None,
                    distributed_sampler_cls=None, excluded=None, included=None, load_strategy=None,
                    lr_scheduler_cls=None, lr_scheduler_args=None, find_unused_parameters=False,
                    sampler_seed: int = 0, **kwargs):
    """Returns ``(status, AutoAccelerateResult, Strategy)``."""
    dev = _device()
    world = int(os.getenv("WORLD_SIZE", "1")) if not dist.is_initialized() else dist.get_world_size()
    if isinstance(load_strategy, str) and load_strategy == "search":
        # dry-run search (atorch/auto_search.py): needs a model factory + a sample batch
        from .auto_search import search_strategy

        load_strategy, report = search_strategy(kwargs["model_fn"], optim_func, optim_args or {},
                                                kwargs["sample_batch"], loss_func,
                                                max_trials=kwargs.get("max_trials"),
                                                model_input_format=model_input_format)
    elif isinstance(load_strategy, str) and load_strategy == "engine":
        # acceleration-engine service (atorch/engine/): analyse, tune and dry
        # run candidate strategies across all ranks, keep the fastest
        from .engine.worker import search as engine_search

        sample = kwargs.get("sample_batch")
        if sample is None and dataset is not None:
            bs = max(1, (dataloader_args or {}).get("batch_size", 1) // max(1, world))
            sample = next(iter(torch.utils.data.DataLoader(dataset, batch_size=bs)))
        load_strategy = engine_search(model, optim_func, optim_args, loss_func, sample,
                                      model_fn=kwargs.get("model_fn"), model_input_format=model_input_format,
                                      included=included, excluded=excluded, time_limit=kwargs.get("time_limit"),
                                      load_strategy=kwargs.get("engine_load_strategy"),
                                      verbose=kwargs.get("verbose", False),
                                      warmup=int(os.getenv("DWAMD_DRYRUN_WARMUP", "2")),
                                      steps=int(os.getenv("DWAMD_DRYRUN_STEPS", "3")))
        included = excluded = None  # already applied by the engine's planner
    strategy =Strategy.from_spec(load_strategy) if load_strategy is not None else plan_strategy(model, world)
    if excluded:
        strategy = Strategy([o for o in strategy.opts if o[0] not in excluded])
    if included:
        have = set(strategy.names())
        strategy = Strategy.from_spec(strategy.opts + [(n, None) for n in included if n not in have])
    if world > 1 and "mixed_parallel" in strategy.names():
        mcfg = _mixed_cfg(strategy.config("mixed_parallel"))
        sized_elsewhere = "parallel_mode" in strategy.names() or adist.parallel_config() is not None
        if mcfg.get("auto") or not (mcfg.get("tensor") or mcfg.get("pipeline") or sized_elsewhere):
            # automatic tensor x pipeline x data sizing (atorch/shard_planner.py)
            from .shard_planner import Hardware, plan_3d

            plans = plan_3d(model, world, seq=int(mcfg.get("seq_len", 4096)),
                            micro_batch=int(mcfg.get("micro_batch", 1)), global_batch=mcfg.get("global_batch"),
                            hw=Hardware(gpus_per_node=int(mcfg.get("gpus_per_node", min(8, world)))),
                            act_ckpt=bool(mcfg.get("act_ckpt", False)))
            best = next((x for x in plans if x.feasible), plans[0])
            mcfg = dict(mcfg, **best.as_strategy_cfg())
            mcfg.pop("auto", None)
            logger.info(f"mixed_parallel auto plan: tensor {best.tensor} x pipeline {best.pipeline} x data "
                        f"{best.data} ({best.chunks} micro-batches), ~{best.mem_gb} GB / GPU, est. "
                        f"{best.step_s:.3f} s / step; runner-up "
                        f"{[(x.tensor, x.pipeline, x.data) for x in plans[1:3]]}")
            strategy = Strategy.from_spec([(n, mcfg if n == "mixed_parallel" else c) for n, c in strategy.opts])
    if world > 1 and "mixed_parallel" in strategy.names() and "parallel_mode" not in strategy.names():
        mcfg = _mixed_cfg(strategy.config("mixed_parallel"))
        t, p = int(mcfg.get("tensor", 1)), int(mcfg.get("pipeline", 1))
        dims = [("tensor", t), ("pipeline", p), ("data", int(mcfg.get("data", world // max(1, t * p))))]
        strategy = Strategy.from_spec([("parallel_mode", (dims, None))] + strategy.opts)
    if world > 1 and "parallel_mode" not in strategy.names():
        strategy = Strategy.from_spec([("parallel_mode", None)] + strategy.opts)
    if world > 1 and not {"ddp", "fsdp", "zero2", "zero1", "flat_fsdp", "flat_zero2"} & set(strategy.names()):
        strategy = Strategy.from_spec(strategy.opts + [("ddp", None)])
    if "zero1" in strategy.names() and "ddp" not in strategy.names():
        strategy = Strategy.from_spec(strategy.opts + [("ddp", None)])

    ctx: Dict[str, Any] = {"model": model, "find_unused_parameters": find_unused_parameters,
                           "tp_like": bool({"tensor_parallel", "sequence_parallel", "mixed_parallel"}
                                           & set(strategy.names()))}
    for name, cfg in strategy.opts:
        if name == "parallel_mode":
            APPLY[name](ctx, cfg)
            if (dev.type == "cuda" and not {"pipeline_parallel", "mixed_parallel"} & set(strategy.names())
                    and not _meta_model(ctx["model"])):
                ctx["model"] = ctx["model"].to(dev)  # a pipeline moves only its own stage later
            continue
        APPLY[name](ctx, cfg)
    model = ctx["model"]
    if _meta_model(model):
        raise RuntimeError("a meta-device model needs the fsdp / zero2 strategy (it materialises per shard)")
    if dev.type == "cuda" and not ctx.get("meta_init"):
        model = model.to(dev)
    if ctx.get("amp_dtype") is not None and not ctx.get("fsdp") and not ctx.get("pipeline"):
        model = _AutocastModule(model, ctx["amp_dtype"])

    optim = None
    if optim_func is not None:
        params = optim_param_func(model) if optim_param_func else model.parameters()
        args = dict(optim_args or {})
        if kwargs.get("fused_optimizer", True):
            # torch AdamW/Adam and ATorch AGD -> one multi-tensor HIP launch
            # over the (DTensor-sharded) parameters, fp32 masters for bf16 ones
            from ..optimizers.multi_tensor import fused_equivalent

            fcls, fargs = fused_equivalent(optim_func, args)
            if fcls is not None:
                params = list(params)
                n_groups = len(params) if params and isinstance(params[0], dict) else 1
                if n_groups <= 16:
                    optim_func, args = fcls, fargs
                    logger.info(f"optimizer: {fcls.__name__} (multi-tensor HIP kernel)")
        if ctx.get("flat_fsdp") is not None:
            optim = _flat_optimizer(ctx["flat_fsdp"], optim_func, args)
        elif ctx.get("zero1"):
            from torch.distributed.optim import ZeroRedundancyOptimizer

            optim = ZeroRedundancyOptimizer(params, optimizer_class=optim_func, process_group=ctx.get("dp_group"),
                                            **args)
        else:
            optim = optim_func(params, **args)
        if ctx.get("local_sgd") and optim is not None:
            from .local_sgd import GTAReducer, HSDPLocalSGD, LinearReducer

            rg, lcfg = ctx["local_sgd"]
            red = None
            if lcfg.get("reducer") == "gta":
                red = GTAReducer(rg, consensus_method=lcfg.get("consensus_method", "sum"),
                                 sparsification_method=lcfg.get("sparsification_method"),
                                 normalize=lcfg.get("normalize", True), density=lcfg.get("density", 1.0))
            elif lcfg.get("reducer") in (None, "linear"):
                red = LinearReducer(rg)
            optim = HSDPLocalSGD(model, optim, rg, sync_interval=lcfg.get("local_sgd_sync_interval", 1),
                                 warmup_steps=lcfg.get("local_sgd_warmup_steps", 0),
                                 outer_optim_class=lcfg.get("outer_optim_class"),
                                 outer_optim_kwargs=lcfg.get("outer_optim_kwargs"), reducer=red,
                                 cpu_offload=lcfg.get("outer_optim_cpu_offload", False))
            logger.info(f"fsdp: local SGD over the replicate dimension (sync every "
                        f"{optim.sync_interval} steps after {optim.warmup_steps} warm-up steps)")
    if ctx.get("optim_in_backward") and optim is not None:
        from ..optimizers.in_backward import install

        if install(model, optim) is not None:
            logger.info("fsdp: optimizer update per FSDP unit inside the backward")
    if ctx.get("moe_ddp") is not None and optim is not None:
        ctx["moe_ddp"].attach_optimizer(getattr(optim, "optimizer", optim))
    if ctx.get("fp8") and optim is not None:
        # delayed scaling: the step's recorded amaxes become the next scales
        from ..ops.fp8 import fp8_update

        inner = getattr(optim, "optimizer", optim)
        if hasattr(inner, "register_step_post_hook"):
            inner.register_step_post_hook(lambda *_a, **_k: fp8_update())
        else:
            logger.warning("fp8: optimizer has no step hooks; call ops.fp8.fp8_update() after each step")
    sched = lr_scheduler_cls(optim, **(lr_scheduler_args or {})) if (lr_scheduler_cls and optim) else None

    dp_rank, dp_size = _data_partition(ctx)
    _PARTITION[:] = [dp_rank, dp_size]
    dataloader = None
    if dataset is not None:
        dl_args = dict(dataloader_args or {})
        if dp_size > 1:
            bs = dl_args.get("batch_size", 1)
            dl_args["batch_size"] = max(1, bs // dp_size)  # batch_size is the global batch
            cls = distributed_sampler_cls
            if cls is None:
                from ..trainer.elastic import ElasticDistributedSampler as cls
            dl_args["sampler"] = cls(dataset, num_replicas=dp_size, rank=dp_rank,
                                     shuffle=dl_args.pop("shuffle", True), seed=sampler_seed)
        dataloader = torch.utils.data.DataLoader(dataset, **dl_args)

    if loss_func is not None and ctx.get("amp_dtype") is not None:
        # the loss runs under the same autocast as the forward (reference
        # amp_optimization.py:73-78): mixed bf16 outputs / fp32 labels
        loss_func = _autocast_fn(loss_func, ctx["amp_dtype"])
    prep = prepare_input or _default_prepare_input
    if ctx.get("sp") and ctx["sp"][2] is not None:
        sp_size, sp_rank, sp_fn = ctx["sp"]
        base_prep = prep

        def prep(data, device, _b=base_prep):  # noqa: F811
            return sp_fn(_b(data, device), sp_size, sp_rank)
    result = AutoAccelerateResult(model=model, optim=optim, dataloader=dataloader, loss_func=loss_func,
                                  prepare_input=prep, lr_scheduler=sched,
                                  args={"model_input_format": model_input_format,
                                        "grad_scaler": ctx.get("grad_scaler"), "device": dev,
                                        "amp_dtype": ctx.get("amp_dtype")})
    return True, result, strategy


def model_transform(model: nn.Module, strategy) -> nn.Module:
    """Apply a strategy to a model only (no optimizer / data)."""
    _ok, res, _s = auto_accelerate(model, load_strategy=strategy)
    return res.model
