"""Executor: owns the task queue of one acceleration and hands tasks to the
training processes that poll the engine.

* ONE_PROCESS tasks (ANALYSE, TUNE) go to whichever process asks first;
* ALL_PROCESS tasks (SETUP_PARALLEL_GROUP, DRYRUN, FINISH/FAIL) are handed
  out only once every process is idle, then to each process once; the task
  completes when all have reported (process 0's result is kept -- the dry
  runner already reduced the step time to the slowest rank);
* a SETUP_PARALLEL_GROUP task whose parallel mode is the one already set up
  is dropped, so dry runs sharing a parallel mode reuse its RCCL
  communicators;
* when nothing is queued or running, the planner and then the selected SG
  algorithms are asked for new strategies; once they are exhausted (or the
  time limit passed) a FINISH task with the fastest dry-run strategy (FAIL if
  none succeeded) ends the acceleration.

Parity: reference ``atorch/atorch/auto/engine/executor.py`` (``Executor``,
``ProcessStatus``, ``get_task`` / ``report_task_result`` /
``generate_tasks_if_needed``).
"""

import threading
import time
from typing import Any, Dict, List, Optional

from ...common.log import logger
from .planner import HBM_BYTES, Planner, SGAlgorithmLibrary
from .strategy import OptimizationMethodLibrary, StrategyStatus, StrategyTable, parallel_mode_of
from .task import ProcessMode, Task, TaskStatus, TaskType


class Executor:
    def __init__(self, device_context: Dict[str, Any], included_opts=None, excluded_opts=None,
                 time_limit: Optional[float] = None, load_strategy=None, verbose: bool = False):
        self.ctx = dict(device_context or {})
        self.total_process = max(1, int(self.ctx.get("node_num", 1)) * int(self.ctx.get("nproc_per_node", 1)))
        self.hbm_bytes = int(self.ctx.get("hbm_bytes", HBM_BYTES))
        self.lib = OptimizationMethodLibrary()
        self.strategies = StrategyTable(self.lib)
        self.algo_lib = SGAlgorithmLibrary()
        self.planner = Planner(self.lib, self.strategies, self.ctx, load_strategy, included_opts, excluded_opts)
        self.analysis: Dict[str, Any] = {}
        self.time_limit = time_limit
        self.verbose = verbose
        self.start_time = time.time()
        self.end_time: Optional[float] = None
        self._lock = threading.RLock()
        self.tasks: Dict[int, Task] = {}
        self.pending: List[int] = []
        self.unfinished = 0
        self.busy: List[Optional[int]] = [None] * self.total_process   # task id per process
        self.assigning: Optional[int] = None
        self.reported: Dict[int, int] = {}
        self.current_parallel_mode = None
        self.terminate_id: Optional[int] = None
        self.in_planner = True
        self.algos: List[str] = []
        self.algo_idx = 0
        with self._lock:
            self._refill()

    # ------------------------------------------------------------ tasks
    def add_tasks(self, tasks: List[Task]):
        for t in tasks:
            t.task_id = len(self.tasks)
            self.tasks[t.task_id] = t
            self.pending.append(t.task_id)
            self.unfinished += 1
            if t.strategy_id >= 0:
                self.strategies.bind(t.strategy_id, t.task_id)
            if t.task_type in (TaskType.FINISH, TaskType.FAIL):
                self.terminate_id = t.task_id

    def _tasks_for(self, s_id: int) -> List[Task]:
        info = self.strategies[s_id]
        setup = Task(TaskType.SETUP_PARALLEL_GROUP, parallel_mode_of(info.strategy), process_mode=ProcessMode.ALL)
        if info.status == StrategyStatus.INIT:
            work = Task(TaskType.TUNE, info.strategy, strategy_id=s_id, process_mode=info.tune_mode)
        else:
            work = Task(TaskType.DRYRUN, info.strategy, strategy_id=s_id, process_mode=ProcessMode.ALL)
        return [setup, work]

    def _out_of_time(self) -> bool:
        return self.time_limit is not None and time.time() - self.start_time > self.time_limit

    def _refill(self):
        if self.terminate_id is not None or self.pending:
            return
        for _ in range(10000):
            s_id = self.strategies.next_inactive()
            if s_id is not None and not self._out_of_time():
                self.add_tasks(self._tasks_for(s_id))
                return
            if self.unfinished > 0:
                return  # wait for the running tasks' results
            if self._out_of_time():
                logger.info(f"engine: time limit {self.time_limit}s reached")
                break
            if self.in_planner:
                done, tasks, _n, algos = self.planner.plan(self)
                if tasks:
                    self.add_tasks(tasks)
                    return
                if done:
                    self.in_planner, self.algos = False, list(algos)
                continue
            if self.algo_idx >= len(self.algos):
                break
            algo = self.algo_lib[self.algos[self.algo_idx]]
            if algo is None:
                self.algo_idx += 1
                continue
            done, tasks, n = algo.generate(self)
            if done or (not tasks and n == 0):
                self.algo_idx += 1
            if tasks:
                self.add_tasks(tasks)
                return
        best = self.strategies.best()
        if best is None:
            self.add_tasks([Task(TaskType.FAIL, None, process_mode=ProcessMode.ALL)])
        else:
            self.add_tasks([Task(TaskType.FINISH, best, process_mode=ProcessMode.ALL)])
        self.end_time = time.time()
        logger.info(f"engine: acceleration search done in {self.end_time - self.start_time:.1f}s, "
                    f"{len(self.strategies)} strategies, best {best}")

    def _pop_pending(self) -> Optional[int]:
        while self.pending:
            t_id = self.pending.pop(0)
            t = self.tasks[t_id]
            if t.task_type == TaskType.SETUP_PARALLEL_GROUP and t.info == self.current_parallel_mode:
                t.status = TaskStatus.SUCCEEDED
                self.unfinished -= 1
                continue
            return t_id
        return None

    def get_task(self, process_id: int) -> Task:
        with self._lock:
            task = None
            if self.assigning is None and self.pending and self.busy[process_id] is None:
                t_id = self._pop_pending()
                if t_id is not None:
                    t = self.tasks[t_id]
                    if t.process_mode == ProcessMode.ONE or self.total_process == 1:
                        t.status = TaskStatus.RUNNING
                        self._assign(t_id, process_id)
                        task = t
                    else:
                        t.status = TaskStatus.ASSIGNING
                        self.assigning = t_id
            if task is None and self.assigning is not None:
                t_id = self.assigning
                t = self.tasks[t_id]
                # an ALL_PROCESS task starts once every process is idle
                if process_id not in t.assigned and (t.assigned or all(b is None for b in self.busy)):
                    self._assign(t_id, process_id)
                    task = t
                if len(t.assigned) == self.total_process:
                    t.status = TaskStatus.RUNNING
                    self.assigning = None
            if task is None:
                task = Task(TaskType.WAIT)
            elif self.verbose:
                logger.info(f"engine: process {process_id} <- task {task.task_id} {task.task_type}")
            return task

    def _assign(self, t_id: int, process_id: int):
        self.tasks[t_id].assigned.append(process_id)
        self.busy[process_id] = t_id

    def report_task_result(self, task_id: int, process_id: int, ok: bool, result):
        with self._lock:
            if self.busy[process_id] == task_id:
                self.busy[process_id] = None
            t = self.tasks[task_id]
            if t.process_mode == ProcessMode.ALL and self.total_process > 1:
                self.reported[task_id] = self.reported.get(task_id, 0) + 1
                if process_id == 0:
                    t.result = result
                t.status = TaskStatus.FAILED if not ok else t.status
                if self.reported[task_id] < self.total_process:
                    return
                ok = t.status != TaskStatus.FAILED
                result = t.result
            else:
                t.result = result
            t.status = TaskStatus.SUCCEEDED if ok else TaskStatus.FAILED
            if ok and t.task_type == TaskType.ANALYSE and isinstance(result, dict):
                self.analysis.update(result)
            if t.task_type == TaskType.SETUP_PARALLEL_GROUP:
                self.current_parallel_mode = t.info if ok else None
            self.strategies.task_done(task_id, t.task_type, ok, result)
            self.unfinished -= 1
            if self.verbose:
                logger.info(f"engine: task {task_id} {t.task_type} -> {t.status} ({result})")
            self._refill()

    @property
    def can_be_terminated(self) -> bool:
        return self.terminate_id is not None and len(self.tasks[self.terminate_id].assigned) == self.total_process

    def summary(self) -> List[Dict[str, Any]]:
        return [{"id": i, "strategy": [x[0] for x in s.strategy], "status": s.status,
                 "result": s.dryrun_result} for i, s in self.strategies.infos.items()]
