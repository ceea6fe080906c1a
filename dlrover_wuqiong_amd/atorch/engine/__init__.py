"""ATorch acceleration engine: planner + executor + strategy generation,
served over gRPC from rank 0 to every training process.

Parity: reference ``atorch/atorch/auto/engine/``.
"""

from .executor import Executor
from .planner import BayesOptSG, CombinationSG, Planner, SGAlgorithmLibrary, candidate_space
from .service import AccelerationEngine, EngineClient
from .strategy import OptimizationMethodLibrary, StrategyStatus, StrategyTable
from .task import ProcessMode, Task, TaskStatus, TaskType

__all__ = ["AccelerationEngine", "EngineClient", "Executor", "Planner", "SGAlgorithmLibrary", "CombinationSG",
           "BayesOptSG", "candidate_space", "OptimizationMethodLibrary", "StrategyStatus", "StrategyTable",
           "ProcessMode", "Task", "TaskStatus", "TaskType"]
