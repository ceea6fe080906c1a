"""Optimization-method library and the engine's strategy table.

The library describes every optimization ``auto_accelerate`` can apply
(group, devices, whether it only makes sense distributed, whether it needs
tuning) and prunes against the device context: methods needing the gfx950
HIP kernels are dropped on any other GPU, distributed-only methods on one
process, and strategies whose predicted training state (from the analyser)
cannot fit in HBM are rejected before they cost a dry run.

Parity: reference ``atorch/atorch/auto/engine/optimization_method.py``
(``OptimizationMethod``, ``OptimizationMethodLibrary``) and
``auto/engine/strategy.py`` (``StrategyStatus``, ``StrategyInfoCollection``,
``strategy_duplicate``).
"""

from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ...common.log import logger
from .task import ProcessMode, TaskType

Strategy = List[Tuple[str, Any, bool]]   # [(name, config, tunable)]


@dataclass
class OptimizationMethod:
    name: str
    group: str
    devices: Tuple[str, ...] = ("cpu", "cuda")
    gpu_archs: Optional[Tuple[str, ...]] = None   # None: any GPU
    distributed_only: bool = False
    tunable: bool = False
    process_mode: str = ProcessMode.ONE
    saves_memory: bool = False
    speeds_compute: bool = False
    disabled: bool = False


class OptimizationMethodLibrary:
    GROUPS = {
        "parallel_mode": ["parallel_mode"],
        "amp": ["amp_native", "half"],
        "zero": ["zero1", "zero2", "fsdp"],
        "parallel": ["tensor_parallel", "sequence_parallel", "pipeline_parallel"],
        "module_replace": ["module_replace"],
        "checkpoint": ["checkpoint"],
    }
    # pairs that never go together in one strategy
    INVALID = [{"zero1", "zero2"}, {"zero1", "fsdp"}, {"zero2", "fsdp"}, {"pipeline_parallel", "fsdp"},
               {"pipeline_parallel", "zero2"}, {"pipeline_parallel", "zero1"}]

    def __init__(self):
        m = OptimizationMethod
        self.methods: Dict[str, OptimizationMethod] = {}
        for meth in [
            m("parallel_mode", "parallel_mode"),
            m("amp_native", "amp", speeds_compute=True),
            m("half", "amp", devices=("cuda",), speeds_compute=True, saves_memory=True),
            m("zero1", "zero", distributed_only=True, saves_memory=True),
            m("zero2", "zero", distributed_only=True, saves_memory=True),
            m("fsdp", "zero", distributed_only=True, saves_memory=True),
            m("tensor_parallel", "parallel", distributed_only=True, tunable=True, saves_memory=True),
            m("sequence_parallel", "parallel", distributed_only=True, saves_memory=True),
            m("pipeline_parallel", "parallel", distributed_only=True, tunable=True, saves_memory=True),
            # fused norms / flash attention are gfx950 HIP kernels (CPU runs the reference math)
            m("module_replace", "module_replace", gpu_archs=("gfx950",), speeds_compute=True, saves_memory=True),
            m("checkpoint", "checkpoint", saves_memory=True),
        ]:
            self.methods[meth.name] = meth

    def __getitem__(self, name) -> OptimizationMethod:
        return self.methods[name]

    def names(self, group: Optional[str] = None) -> List[str]:
        return list(self.GROUPS[group]) if group else list(self.methods)

    def enabled(self, name: str) -> bool:
        return name in self.methods and not self.methods[name].disabled

    def disable(self, names: Sequence[str]):
        """Method or group names."""
        for n in names:
            for x in self.GROUPS.get(n, [n]):
                if x in self.methods:
                    self.methods[x].disabled = True

    def prune_for_device(self, ctx: Dict[str, Any]) -> List[str]:
        total = int(ctx.get("node_num", 1)) * int(ctx.get("nproc_per_node", 1))
        has_gpu = int(ctx.get("total_gpu", 0)) > 0
        arch = str(ctx.get("gpu_arch", ""))
        out = []
        for name, meth in self.methods.items():
            if (meth.distributed_only and total == 1) or (not has_gpu and "cpu" not in meth.devices) or \
                    (has_gpu and meth.gpu_archs and not any(arch.startswith(a) for a in meth.gpu_archs)):
                out.append(name)
        self.disable(out)
        return out

    def validate(self, strategy: Strategy) -> Tuple[bool, str]:
        """(valid, process mode of its TUNE task)."""
        names = set()
        mode = ProcessMode.ONE
        for item in strategy:
            if len(item) != 3:
                return False, mode
            name = item[0]
            if not self.enabled(name):
                return False, mode
            names.add(name)
            if self.methods[name].process_mode == ProcessMode.ALL:
                mode = ProcessMode.ALL
        if any(bad <= names for bad in self.INVALID):
            return False, mode
        return True, mode


def parallel_mode_of(strategy: Strategy):
    for name, cfg, _ in strategy:
        if name == "parallel_mode":
            return cfg
    return None


def same_strategy(a: Strategy, b: Strategy) -> bool:
    """Same methods, and the same parallel mode."""
    if sorted(x[0] for x in a) != sorted(x[0] for x in b):
        return False
    return parallel_mode_of(a) == parallel_mode_of(b)


def predicted_state_bytes(strategy: Strategy, analysis: Dict[str, Any], world: int) -> Optional[int]:
    """Per-process bytes of weights + grads + masters + Adam moments implied
    by ``strategy`` (None if the analyser has not run)."""
    sb = analysis.get("state_bytes") if analysis else None
    if not sb:
        return None
    names = [x[0] for x in strategy]
    zero = next((n for n in ("fsdp", "zero2", "zero1") if n in names), "ddp")
    b = sb.get(zero, sb.get("ddp", 0))
    tp = 1
    pm = parallel_mode_of(strategy)
    if pm:
        for dim in pm[0]:
            if dim[0] in ("tensor", "pipeline"):
                tp *= int(dim[1])
    return int(b // max(1, tp))


class StrategyStatus:
    INIT = "INIT"          # has tunable methods not tuned yet
    TUNED = "TUNED"        # ready for a dry run
    SUCCEED = "SUCCEED"    # dry run finished
    FAILED = "FAILED"      # tune or dry run failed


@dataclass
class StrategyInfo:
    strategy: Strategy
    status: str
    tune_mode: str = ProcessMode.ONE
    dryrun_result: Optional[Dict[str, Any]] = None
    baseline: bool = False


class StrategyTable:
    """Every candidate strategy of this acceleration with its status and dry
    run result, plus the task -> strategy mapping."""

    def __init__(self, lib: OptimizationMethodLibrary):
        self.lib = lib
        self.infos: Dict[int, StrategyInfo] = {}
        self.task_owner: Dict[int, int] = {}
        self.open_tasks: Dict[int, List[int]] = {}
        self.baseline_id: Optional[int] = None

    def __len__(self):
        return len(self.infos)

    def __getitem__(self, s_id) -> StrategyInfo:
        return self.infos[s_id]

    def add(self, strategy: Strategy, baseline: bool = False, skip_duplicate: bool = True) -> Optional[int]:
        strategy = [tuple(x) for x in strategy]
        ok, mode = self.lib.validate(strategy)
        if not ok:
            logger.debug(f"engine: invalid strategy {strategy}")
            return None
        if skip_duplicate and any(same_strategy(i.strategy, strategy) for i in self.infos.values()):
            return None
        status = StrategyStatus.INIT if any(t for _, _, t in strategy) else StrategyStatus.TUNED
        s_id = len(self.infos)
        self.infos[s_id] = StrategyInfo(list(strategy), status, mode, baseline=baseline)
        if baseline:
            self.baseline_id = s_id
        return s_id

    def next_inactive(self) -> Optional[int]:
        """A strategy still to tune / dry run with no task in flight."""
        for s_id, info in self.infos.items():
            if info.status in (StrategyStatus.SUCCEED, StrategyStatus.FAILED) or self.open_tasks.get(s_id):
                continue
            return s_id
        return None

    def bind(self, s_id: int, task_id: int):
        self.task_owner[task_id] = s_id
        self.open_tasks.setdefault(s_id, []).append(task_id)

    def task_done(self, task_id: int, task_type: str, ok: bool, result):
        s_id = self.task_owner.get(task_id)
        if s_id is None:
            return
        if task_id in self.open_tasks.get(s_id, []):
            self.open_tasks[s_id].remove(task_id)
        info = self.infos[s_id]
        if not ok:
            info.status = StrategyStatus.FAILED
            info.dryrun_result = result if isinstance(result, dict) else info.dryrun_result
        elif task_type == TaskType.TUNE:
            info.strategy = [tuple(x) for x in result]
            info.status = StrategyStatus.TUNED
        elif task_type == TaskType.DRYRUN:
            info.status = StrategyStatus.SUCCEED
            info.dryrun_result = result

    def finished(self) -> Dict[int, StrategyInfo]:
        return {i: s for i, s in self.infos.items() if s.status in (StrategyStatus.SUCCEED, StrategyStatus.FAILED)}

    def best(self) -> Optional[Strategy]:
        good = [(s.dryrun_result.get("throughput", 0.0), -i, s.strategy) for i, s in self.infos.items()
                if s.status == StrategyStatus.SUCCEED and s.dryrun_result]
        return max(good)[2] if good else None
