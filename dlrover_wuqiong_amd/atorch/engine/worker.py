"""Training-process side of the acceleration engine: poll tasks, run them,
report results, return the chosen strategy.

``auto_accelerate(..., load_strategy="engine")`` calls :func:`search`:
rank 0 starts the :class:`AccelerationEngine`, the port is broadcast, and
every rank loops ``get_task -> run -> report`` until FINISH (the fastest
strategy, then applied to the user's model by ``auto_accelerate``) or FAIL.

Task runners:
  ANALYSE               ``auto_search.analyse_model`` + what the planner prunes on
                        (replaceable modules, TP-able projections, head count)
  SETUP_PARALLEL_GROUP  (re)create the named process groups, unless unchanged
  TUNE                  fill tunable methods: tensor parallel -> the smallest
                        TP degree within one xGMI node (<= 8, divides the heads and
                        the world) whose predicted training state fits HBM
  DRYRUN                ``DryRunner.profile`` on a fresh copy of the model; the step
                        time is reduced to the slowest rank (MAX) and success to the
                        AND over ranks, so every rank reports the same verdict
  WAIT                  sleep briefly and poll again

Parity: reference ``atorch/atorch/auto/accelerate.py:86-232`` (``run_task`` and
the per-type runners) and ``:583-640`` (engine start, port broadcast, task loop).
"""

import copy
import os
import time
from typing import Any, Callable, Dict, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn

from ...common.log import logger
from .. import distributed as adist
from .strategy import Strategy, parallel_mode_of, predicted_state_bytes
from .task import TaskType

_COL = ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj", "c_fc", "fc1", "w1", "w3", "query_key_value")
_HEAD_ATTRS = ("num_attention_heads", "num_heads", "n_head")


def device_context() -> Dict[str, Any]:
    world = dist.get_world_size() if dist.is_initialized() else int(os.getenv("WORLD_SIZE", "1"))
    local = int(os.getenv("LOCAL_WORLD_SIZE", str(world)))
    ctx = {"node_num": max(1, world // max(1, local)), "nproc_per_node": min(local, world), "total_gpu": 0}
    if torch.cuda.is_available():
        props = torch.cuda.get_device_properties(torch.cuda.current_device())
        ctx.update(total_gpu=world, gpu_arch=getattr(props, "gcnArchName", ""), hbm_bytes=int(props.total_memory))
    return ctx


def _num_heads(model: nn.Module) -> Optional[int]:
    cfg = getattr(model, "config", None)
    for src in (cfg, model):
        for a in _HEAD_ATTRS:
            v = getattr(src, a, None) if src is not None else None
            if isinstance(v, int) and v > 0:
                return v
    for m in model.modules():
        for a in _HEAD_ATTRS:
            v = getattr(m, a, None)
            if isinstance(v, int) and v > 0 and not isinstance(m, nn.Linear):
                return v
    return None


def analyse(model: nn.Module, world: int) -> Dict[str, Any]:
    from ..auto_search import analyse_model

    res = analyse_model(model, world)
    types = res["module_types"]
    res["has_module_for_replace"] = bool(
        types.get("LayerNorm", 0) or any("RMSNorm" in t for t in types) or
        getattr(getattr(model, "config", None), "_attn_implementation", None) is not None)
    res["tp_able"] = any(n.rsplit(".", 1)[-1] in _COL for n, m in model.named_modules() if isinstance(m, nn.Linear))
    res["num_heads"] = _num_heads(model)
    return res


def to_spec(strategy: Strategy) -> List:
    """Engine strategy -> ``auto_accelerate`` spec."""
    return [(name, cfg) for name, cfg, _t in strategy]


def tune(strategy: Strategy, analysis: Dict[str, Any], ctx: Dict[str, Any]) -> Optional[Strategy]:
    world = int(ctx.get("node_num", 1)) * int(ctx.get("nproc_per_node", 1))
    out = [list(x) for x in strategy]
    for item in out:
        if not item[2]:
            continue
        if item[0] == "tensor_parallel":
            heads = analysis.get("num_heads") or 0
            hbm = int(ctx.get("hbm_bytes", 288 * 2 ** 30))
            choice = None
            for t in range(2, min(8, int(ctx.get("nproc_per_node", world))) + 1):
                if world % t or (heads and heads % t):
                    continue
                choice = t
                pm = ([("tensor", t), ("data", world // t)], None)
                trial = [(n, pm if n == "parallel_mode" else c, False) for n, c, _ in out]
                pred = predicted_state_bytes(trial, analysis, world)
                if pred is None or pred <= 0.9 * hbm:
                    break
            if choice is None:
                return None
            pm = ([("tensor", choice), ("data", world // choice)], None)
            if not any(x[0] == "parallel_mode" for x in out):
                out.insert(0, ["parallel_mode", pm, False])
            for x in out:
                if x[0] == "parallel_mode":
                    x[1] = pm
        item[2] = False
    return [tuple(x) for x in out]


class _Worker:
    def __init__(self, model: nn.Module, optim_func, optim_args, loss_func, sample_batch, model_fn,
                 model_input_format, warmup: int, steps: int):
        self.model = model
        self.optim_func = optim_func
        self.optim_args = optim_args or {}
        self.loss_func = loss_func
        self.sample_batch = sample_batch
        self.model_fn = model_fn or (lambda: copy.deepcopy(model))
        self.model_input_format = model_input_format
        self.warmup, self.steps = warmup, steps
        self.ctx = device_context()
        self.world = int(self.ctx["node_num"]) * int(self.ctx["nproc_per_node"])
        self.analysis: Dict[str, Any] = {}
        self.mode = None   # parallel mode currently set up

    def setup(self, p_mode) -> bool:
        if p_mode == self.mode and (p_mode is None or adist.parallel_config() is not None):
            return True
        ok = True
        try:
            adist.destroy_parallel_group()
            if p_mode is not None and dist.is_initialized():
                adist.create_parallel_group(p_mode)
            self.mode = p_mode
        except Exception as e:
            logger.error(f"engine: parallel group setup {p_mode} failed: {e}")
            ok = False
        if dist.is_initialized():
            dist.barrier()
        return ok

    def dryrun(self, strategy: Strategy):
        from ..auto_search import DryRunner

        r = DryRunner.profile(self.model_fn, to_spec(strategy), self.optim_func, self.optim_args,
                              self.sample_batch, self.loss_func, warmup=self.warmup, steps=self.steps,
                              model_input_format=self.model_input_format, keep_groups=True)
        step_time, ok = (r.step_time, r.ok)
        if dist.is_initialized() and dist.get_world_size() > 1:
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
            t = torch.tensor([step_time if ok else float("inf"), 0.0 if ok else 1.0], dtype=torch.float64,
                             device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            step_time, ok = float(t[0]), float(t[1]) == 0.0
        if not ok:
            return False, {"error": r.error or "failed on another rank"}
        bs = r.throughput * r.step_time  # samples per step over the data group
        return True, {"throughput": bs / step_time, "step_time": step_time, "max_memory_bytes": r.max_memory_bytes}

    def run(self, task):
        tt = task.task_type
        if tt == TaskType.ANALYSE:
            self.analysis = analyse(self.model, self.world)
            return True, self.analysis
        if tt == TaskType.SETUP_PARALLEL_GROUP:
            return self.setup(task.info), None
        if tt == TaskType.TUNE:
            if not self.analysis:  # the ANALYSE task may have run on another process
                self.analysis = analyse(self.model, self.world)
            res = tune(task.info, self.analysis, self.ctx)
            return res is not None, res
        if tt == TaskType.DRYRUN:
            return self.dryrun(task.info)
        return False, None


def search(model: nn.Module, optim_func, optim_args=None, loss_func: Optional[Callable] = None, sample_batch=None,
           model_fn=None, model_input_format=None, included=None, excluded=None, time_limit=None,
           load_strategy=None, verbose: bool = False, warmup: int = 2, steps: int = 3,
           poll_interval: float = 0.05):
    """Run the engine-driven strategy search; returns the chosen
    ``auto_accelerate`` spec (raises if no strategy could run)."""
    from .service import AccelerationEngine, EngineClient

    if int(os.getenv("WORLD_SIZE", "1")) > 1 and not dist.is_initialized():
        adist.init_distributed("nccl")
    rank = dist.get_rank() if dist.is_initialized() else 0
    engine = None
    port = 0
    if rank == 0:
        engine = AccelerationEngine(device_context(), included_opts=included, excluded_opts=excluded,
                                    time_limit=time_limit, load_strategy=load_strategy, verbose=verbose)
        port = engine.start_service(0)
    if dist.is_initialized() and dist.get_world_size() > 1:
        box = [port]
        dist.broadcast_object_list(box, src=0)
        port = box[0]
    client = EngineClient(os.getenv("MASTER_ADDR", "127.0.0.1"), port, process_id=rank)
    worker = _Worker(model, optim_func, optim_args, loss_func, sample_batch, model_fn, model_input_format,
                     warmup, steps)
    try:
        while True:
            task = client.get_task()
            if task.task_type == TaskType.WAIT:
                time.sleep(poll_interval)
                continue
            if task.task_type in (TaskType.FINISH, TaskType.FAIL):
                if engine is not None:
                    if verbose:
                        logger.info(f"engine summary: {engine.executor.summary()}")
                    engine.tear_down()
                if task.task_type == TaskType.FAIL:
                    raise RuntimeError("acceleration engine found no strategy that runs")
                best = task.info
                # the final model is built under the winning strategy's parallel mode
                if parallel_mode_of(best) != worker.mode:
                    adist.destroy_parallel_group()
                logger.info(f"engine: selected strategy {[x[0] for x in best]}")
                return to_spec(best)
            try:
                ok, result = worker.run(task)
            except Exception as e:  # a failing task is a result, not a crash
                logger.error(f"engine task {task.task_type} failed: {e}")
                ok, result = False, None
            client.report_task_result(task, ok, result)
    finally:
        client.close()
        if engine is not None and engine.server is not None:
            engine.tear_down(force=True)
