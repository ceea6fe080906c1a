"""Strategy search for ``auto_accelerate``: model analyser, dry runner and
a candidate search (exhaustive, or Bayesian optimisation over the candidate
index space when the space is large).

    best, report = search_strategy(lambda: build_model(), torch.optim.AdamW, {"lr": 1e-4},
                                   sample_batch=batch, loss_func=loss_fn, max_trials=6)
    status, result, strategy = auto_accelerate(build_model(), torch.optim.AdamW,
                                               load_strategy=best, ...)

* ``analyse_model``: parameter count, repeated block class, per-type module
  counts and the training-state bytes each strategy implies (weights, grads,
  fp32 masters, Adam moments; sharded over the data group for ZeRO/FSDP).
* ``DryRunner.profile``: builds a fresh model, applies a strategy through
  ``auto_accelerate``, runs ``warmup`` + ``steps`` optimizer steps on a
  sample batch and returns throughput (samples/s over the data group), peak
  device memory and the step time; a failure (e.g. OOM) is a result, not a
  crash.
* ``search_strategy``: candidates = data-parallel mode (ddp / zero1 / zero2 /
  fsdp) x activation checkpointing x bf16 autocast (+ module_replace); the
  analyser prunes candidates that cannot fit 288 GB of HBM; the rest are dry
  run (all of them, or ``max_trials`` picked by GP-EI over their index
  features) and the fastest that fits wins.

Parity: ATorch ``atorch/auto/analyser/analyser.py``, ``auto/dry_runner/
dry_runner.py`` (``DryRunner.profile`` -> throughput / max_gpu_memory /
data_latency_percentage), ``auto/engine/{planner,strategy,sg_algo}`` (the
strategy generation + BO search of the acceleration engine).
"""

import copy
import itertools
import os
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ..common.log import logger

HBM_BYTES = 288 * 2 ** 30


def analyse_model(model: nn.Module, world: int = 1) -> Dict[str, Any]:
    n = sum(p.numel() for p in model.parameters())
    trainable = sum(p.numel() for p in model.parameters() if p.requires_grad)
    types: Dict[str, int] = {}
    for m in model.modules():
        types[type(m).__name__] = types.get(type(m).__name__, 0) + 1
    from .auto_accelerate import _decoder_layer_classes

    blocks = [c.__name__ for c in _decoder_layer_classes(model)]
    # bytes / parameter: bf16 weight 2 + grad 2..4 + fp32 master 4 + Adam 8
    per_param = {"ddp": 2 + 4 + 4 + 8, "zero1": 2 + 4 + (4 + 8) / world, "zero2": 2 + (4 + 4 + 8) / world,
                 "fsdp": (2 + 4 + 4 + 8) / world}
    return {"params": n, "trainable_params": trainable, "module_types": types, "block_classes": blocks,
            "state_bytes": {k: int(v * trainable) for k, v in per_param.items()}}


@dataclass
class DryRunResult:
    strategy: List[Any]
    ok: bool
    throughput: float = 0.0
    step_time: float = 0.0
    max_memory_bytes: int = 0
    error: str = ""


@dataclass
class SearchReport:
    analysis: Dict[str, Any]
    results: List[DryRunResult] = field(default_factory=list)
    pruned: List[List[Any]] = field(default_factory=list)


class DryRunner:
    @staticmethod
    def profile(model_fn: Callable[[], nn.Module], strategy: List[Any], optim_func, optim_args: Dict,
                sample_batch, loss_func: Callable, warmup: int = 2, steps: int = 3,
                model_input_format: Optional[str] = None, keep_groups: bool = False) -> DryRunResult:
        from .auto_accelerate import auto_accelerate

        dev_cuda = torch.cuda.is_available()
        try:
            if dev_cuda:
                torch.cuda.empty_cache()
                torch.cuda.reset_peak_memory_stats()
            ok, res, _s = auto_accelerate(model_fn(), optim_func, optim_args=optim_args,
                                          load_strategy=copy.deepcopy(strategy),
                                          model_input_format=model_input_format)
            model, opt = res.model, res.optim
            dev = res.args["device"]
            batch = res.prepare_input(sample_batch, dev)
            bs = (batch[0] if isinstance(batch, (list, tuple)) else
                  next(iter(batch.values())) if isinstance(batch, dict) else batch).shape[0]

            def step():
                if model_input_format == "unpack_dict":
                    out = model(**batch)
                elif model_input_format == "unpack_sequence":
                    out = model(*batch)
                else:
                    out = model(batch)
                loss = loss_func(batch, out)
                loss.backward()
                opt.step()
                opt.zero_grad(set_to_none=True)

            for _ in range(warmup):
                step()
            if dev_cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            if dev_cuda:
                torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            dp = _data_parallel_size()
            mem = torch.cuda.max_memory_allocated() if dev_cuda else 0
            del model, opt, res
            return DryRunResult(strategy, True, throughput=bs * dp / dt, step_time=dt, max_memory_bytes=mem)
        except Exception as e:  # OOM or an inapplicable strategy is a data point
            logger.warning(f"dry run of {strategy} failed: {e}")
            return DryRunResult(strategy, False, error=repr(e))
        finally:
            from . import distributed as adist

            # each candidate re-creates its parallel groups (the engine
            # keeps them across dry runs sharing a parallel mode)
            if not keep_groups and adist.parallel_config() is not None:
                adist.destroy_parallel_group()


def _data_parallel_size() -> int:
    """Ranks reading distinct batches: data x zero groups (tensor /
    pipeline ranks of one replica share a batch)."""
    from . import distributed as adist

    if not dist.is_initialized():
        return 1
    if adist.parallel_config() is None:
        return dist.get_world_size()
    n = 1
    for name in ("data", "zero"):
        g = adist.parallel_group(name)
        if g is not None:
            n *= dist.get_world_size(g)
    return n


def candidate_strategies(world: int, include_fsdp: bool = True) -> List[List[Any]]:
    modes = ["ddp", "zero1"] + (["zero2", "fsdp"] if include_fsdp and world > 1 else [])
    if world == 1:
        modes = [None]
    out = []
    for mode, ckpt, amp in itertools.product(modes, (False, True), (True, False)):
        s: List[Any] = ["parallel_mode", "module_replace"]
        if amp:
            s.append(("amp_native", {"dtype": torch.bfloat16}))
        if ckpt:
            s.append("checkpoint")
        if mode:
            s.append(mode)
        out.append(s)
    return out


def _features(s: List[Any]) -> List[float]:
    names = [x if isinstance(x, str) else x[0] for x in s]
    return [float("amp_native" in names), float("checkpoint" in names),
            float(any(n in ("zero2", "fsdp") for n in names)), float("zero1" in names or "fsdp" in names)]


def search_strategy(model_fn: Callable[[], nn.Module], optim_func, optim_args: Dict, sample_batch,
                    loss_func: Callable, max_trials: Optional[int] = None, hbm_bytes: int = HBM_BYTES,
                    model_input_format: Optional[str] = None, warmup: int = 1, steps: int = 2):
    world = dist.get_world_size() if dist.is_initialized() else int(os.environ.get("WORLD_SIZE", "1"))
    analysis = analyse_model(model_fn(), world)
    report = SearchReport(analysis)
    cands = []
    for s in candidate_strategies(world):
        names = [x if isinstance(x, str) else x[0] for x in s]
        mode = next((n for n in names if n in analysis["state_bytes"]), "ddp")
        if analysis["state_bytes"][mode] > 0.9 * hbm_bytes:
            report.pruned.append(s)
            continue
        cands.append(s)
    if max_trials is None or max_trials >= len(cands):
        order = list(range(len(cands)))
        bo = None
    else:
        from ..brain.hpsearch import BayesianOptimizer, RunResult

        order, bo = [], (BayesianOptimizer, RunResult)
    results: Dict[int, DryRunResult] = {}

    def run(i):
        r = DryRunner.profile(model_fn, cands[i], optim_func, optim_args, sample_batch, loss_func,
                              warmup=warmup, steps=steps, model_input_format=model_input_format)
        results[i] = r
        report.results.append(r)

    if bo is None:
        for i in order:
            run(i)
    else:
        BO, RR = bo
        feats = [_features(c) for c in cands]
        run(0)
        run(len(cands) - 1)
        while len(results) < max_trials:
            hist = [[RR(parameters=tuple(feats[i]), reward=(r.throughput if r.ok else 0.0))
                     for i, r in results.items()]]
            prop = BO([[0.0, 1.0]] * len(feats[0]), hist, 1, seed=len(results)).optimize()[0].parameters
            # nearest untried candidate to the proposal
            left = [i for i in range(len(cands)) if i not in results]
            if not left:
                break
            i = min(left, key=lambda j: sum((a - b) ** 2 for a, b in zip(feats[j], prop)))
            run(i)
    good = [r for r in results.values() if r.ok and r.max_memory_bytes <= hbm_bytes]
    if not good:
        raise RuntimeError(f"no strategy ran successfully: {[r.error for r in results.values()]}")
    best = max(good, key=lambda r: r.throughput)
    logger.info(f"strategy search: best {best.strategy} at {best.throughput:.1f} samples/s "
                f"({len(results)} dry runs, {len(report.pruned)} pruned)")
    return best.strategy, report
