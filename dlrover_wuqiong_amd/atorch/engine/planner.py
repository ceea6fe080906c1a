"""Planner and strategy-generation (SG) algorithms of the acceleration engine.

Planner stages: device prune (at construction) -> ANALYSE task (model size,
block classes, replaceable modules, per-strategy training-state bytes) ->
baseline strategy (plain data parallel) -> memory/analysis prune + algorithm
selection.  The candidate space is zero mode x bf16 autocast x activation
checkpointing x module_replace x tensor parallel; candidates whose predicted
training state exceeds 90 % of HBM (288 GB on MI355X) never get dry run.

SG algorithms:
  * ``combination_sg`` -- every surviving candidate, once (small spaces);
  * ``bo_sg``          -- sequential GP-EI (``brain/hpsearch.py``) over the
    candidates' feature vectors, one proposal per call, stopping after
    ``max_iter`` trials or ``patience`` trials without improvement.

Parity: reference ``atorch/atorch/auto/engine/planner.py`` (``Planner``,
stages BASIC_PRUNE/ANALYSE/BASELINE_STRATEGY/SELECT_ALGO) and
``auto/engine/sg_algo/{combination_sg,bayes_opt_sg,sg_algo_lib}.py``.
"""

import itertools
import os
from typing import Any, Dict, List, Optional, Tuple

import torch

from ...common.log import logger
from .strategy import OptimizationMethodLibrary, Strategy, StrategyStatus, StrategyTable, predicted_state_bytes
from .task import Task, TaskType

HBM_BYTES = 288 * 2 ** 30


def data_parallel(world: int) -> Tuple[str, Any, bool]:
    return ("parallel_mode", ([("data", world)], None), False)


def candidate_space(lib: OptimizationMethodLibrary, world: int, analysis: Dict[str, Any],
                    hbm_bytes: int = HBM_BYTES) -> List[Strategy]:
    zeros: List[Optional[str]] = [None]
    if world > 1:
        zeros += [z for z in ("zero1", "zero2", "fsdp") if lib.enabled(z)]
    amps = [False, True] if lib.enabled("amp_native") else [False]
    ckpts = [False, True] if lib.enabled("checkpoint") and analysis.get("block_classes") else [False]
    mrs = [False, True] if lib.enabled("module_replace") and analysis.get("has_module_for_replace") else [False]
    tps = [False, True] if world > 1 and lib.enabled("tensor_parallel") and analysis.get("tp_able") else [False]
    out = []
    for z, amp, ck, mr, tp in itertools.product(zeros, amps, ckpts, mrs, tps):
        s: Strategy = [data_parallel(world)] if world > 1 else []
        if mr:
            s.append(("module_replace", None, False))
        if amp:
            s.append(("amp_native", {"dtype": torch.bfloat16}, False))
        if tp:
            s.append(("tensor_parallel", None, True))
        if ck:
            s.append(("checkpoint", None, False))
        if z:
            s.append((z, None, False))
        if tp and z in ("zero1",):
            continue  # ZeRO-1 over a TP-sharded (DTensor) model is not supported
        # tensor parallel shards the state by up to 8 (one xGMI-connected node)
        pred = predicted_state_bytes(s, analysis, world)
        if pred is not None and tp:
            pred //= min(8, world)
        if pred is not None and pred > 0.9 * hbm_bytes:
            continue
        out.append(s)
    return out


def features(s: Strategy) -> List[float]:
    names = {x[0] for x in s}
    zero = 1.0 if "fsdp" in names else 2 / 3 if "zero2" in names else 1 / 3 if "zero1" in names else 0.0
    return [zero, float("amp_native" in names), float("checkpoint" in names), float("module_replace" in names),
            float("tensor_parallel" in names)]


class SGAlgorithm:
    name = "sg"

    def __init__(self):
        self.is_done = False

    def generate(self, executor) -> Tuple[bool, Optional[List[Task]], int]:
        """-> (is_done, tasks, number of new strategies)."""
        raise NotImplementedError


class CombinationSG(SGAlgorithm):
    name = "combination_sg"

    def generate(self, executor):
        if self.is_done:
            return True, None, 0
        n = 0
        for s in candidate_space(executor.lib, executor.total_process, executor.analysis, executor.hbm_bytes):
            if executor.strategies.add(s) is not None:
                n += 1
        self.is_done = True
        return True, None, n


class BayesOptSG(SGAlgorithm):
    name = "bo_sg"

    def __init__(self, max_iter: int = 30, patience: int = 8, random_sample: int = 2, seed: int = 0):
        super().__init__()
        self.max_iter = int(os.getenv("DWAMD_BO_MAX_ITER", max_iter))
        self.patience = int(os.getenv("DWAMD_BO_PATIENCE", patience))
        self.random_sample = int(os.getenv("DWAMD_BO_RANDOM_SAMPLE", random_sample))
        self.seed = seed
        self.trials = 0

    def _stale(self, table: StrategyTable) -> bool:
        """``patience`` finished trials in a row without a new best."""
        best, since = 0.0, 0
        for info in table.finished().values():
            tp = (info.dryrun_result or {}).get("throughput", 0.0) if info.status == StrategyStatus.SUCCEED else 0
            if tp > best:
                best, since = tp, 0
            else:
                since += 1
        return since >= self.patience

    def generate(self, executor):
        import numpy as np

        from ...brain.hpsearch import BayesianOptimizer, RunResult

        if self.is_done:
            return True, None, 0
        table = executor.strategies
        cands = candidate_space(executor.lib, executor.total_process, executor.analysis, executor.hbm_bytes)
        left = [c for c in cands if not any(_same_methods(c, i.strategy) for i in table.infos.values())]
        if not left or self.trials >= self.max_iter or self._stale(table):
            self.is_done = True
            return True, None, 0
        rng = np.random.default_rng(self.seed + self.trials)
        if self.trials < self.random_sample:
            pick = left[int(rng.integers(len(left)))]
        else:
            hist = [RunResult(parameters=tuple(features(i.strategy)),
                              reward=float((i.dryrun_result or {}).get("throughput", 0.0))
                              if i.status == StrategyStatus.SUCCEED else 0.0)
                    for i in table.finished().values()]
            dim = len(features(left[0]))
            prop = BayesianOptimizer([[0.0, 1.0]] * dim, [hist], 1, seed=self.seed + self.trials).optimize()
            target = np.array(prop[0].parameters)
            pick = min(left, key=lambda c: float(((np.array(features(c)) - target) ** 2).sum()))
        self.trials += 1
        n = 1 if table.add(pick) is not None else 0
        return False, None, n


def _same_methods(a: Strategy, b: Strategy) -> bool:
    # a tuned TP strategy rewrote its parallel mode: compare method names only
    return sorted(x[0] for x in a) == sorted(x[0] for x in b)


class SGAlgorithmLibrary:
    def __init__(self):
        self.algorithms: Dict[str, SGAlgorithm] = {a.name: a for a in (CombinationSG(), BayesOptSG())}

    def __getitem__(self, name) -> Optional[SGAlgorithm]:
        return self.algorithms.get(name)


class PlannerStage:
    ANALYSE = 0
    BASELINE = 1
    SELECT = 2
    DONE = 3


class Planner:
    def __init__(self, lib: OptimizationMethodLibrary, strategies: StrategyTable, device_context: Dict[str, Any],
                 load_strategy: Optional[Strategy] = None, included_opts=None, excluded_opts=None,
                 max_exhaustive: Optional[int] = None):
        self.lib = lib
        self.strategies = strategies
        self.ctx = device_context or {}
        self.load_strategy = load_strategy
        self.included = list(included_opts or [])
        self.max_exhaustive = int(os.getenv("DWAMD_ENGINE_MAX_EXHAUSTIVE", max_exhaustive or 12))
        self.total_process = int(self.ctx.get("node_num", 1)) * int(self.ctx.get("nproc_per_node", 1))
        self.pruned = lib.prune_for_device(self.ctx)
        if excluded_opts:
            lib.disable(excluded_opts)
        if self.included:
            # only the included methods (and the parallel mode) are searched over
            keep = set(self.included) | {"parallel_mode"}
            lib.disable([n for n in lib.names() if n not in keep])
        self.stage = PlannerStage.ANALYSE
        self.algos: List[str] = []

    def plan(self, executor) -> Tuple[bool, Optional[List[Task]], int, List[str]]:
        """-> (is_done, tasks, new strategies, selected algorithms)."""
        if self.load_strategy is not None:
            n = 1 if self.strategies.add(self.load_strategy, skip_duplicate=False) is not None else 0
            self.stage = PlannerStage.DONE
            return True, None, n, []
        if self.stage == PlannerStage.ANALYSE:
            self.stage = PlannerStage.BASELINE
            return False, [Task(TaskType.ANALYSE, ["analyse_basic"])], 0, []
        if self.stage == PlannerStage.BASELINE:
            self.stage = PlannerStage.SELECT
            base = [data_parallel(self.total_process)] if self.total_process > 1 else []
            pred = predicted_state_bytes(base, executor.analysis, self.total_process)
            if pred is not None and pred > 0.9 * executor.hbm_bytes:
                logger.info("engine: plain data parallel cannot fit HBM; no baseline dry run")
                return False, None, 0, []
            n = 1 if self.strategies.add(base, baseline=True) is not None else 0
            return False, None, n, []
        if self.stage == PlannerStage.SELECT:
            self.stage = PlannerStage.DONE
            space = candidate_space(self.lib, self.total_process, executor.analysis, executor.hbm_bytes)
            self.algos = ["combination_sg"] if len(space) <= self.max_exhaustive else ["bo_sg"]
            logger.info(f"engine: {len(space)} candidate strategies -> {self.algos}")
        return True, None, 0, self.algos
