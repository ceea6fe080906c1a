"""Small master-side services: KV store, named syncs/barriers, training
speed, error routing, diagnosis (hang detection), hyper-parameter strategy.

Parity (reference dlrover/python/master/...):
* ``KVStoreService``        elastic_training/kv_store_service.py:18-32
* ``SyncService``           elastic_training/sync_service.py:26-119
* ``SpeedMonitor``          monitor/speed_monitor.py:43-202
* ``ErrorMonitor``          monitor/error_monitor.py:18-120
* ``DiagnosisManager``      diagnosis/diagnosis.py:27-76 + operator/
                            check_training_hang_operator.py:24-47
* ``SimpleStrategyGenerator`` hyperparams/simple_strategy_generator.py:33-179
"""

import threading
import time
from collections import deque
from typing import Dict, List, Optional, Set, Tuple

from ..common.constants import NodeType, PSClusterVersionType, TrainingExceptionLevel
from ..common.log import logger


class KVStoreService:
    def __init__(self):
        self._lock = threading.Lock()
        self._store: Dict[str, bytes] = {}
        self._cond = threading.Condition(self._lock)

    def set(self, key: str, value: bytes):
        with self._cond:
            self._store[key] = value
            self._cond.notify_all()

    def get(self, key: str) -> bytes:
        with self._lock:
            return self._store.get(key, b"")

    def add(self, key: str, amount: int) -> int:
        with self._cond:
            cur = int(self._store.get(key, b"0") or b"0")
            cur += amount
            self._store[key] = str(cur).encode()
            self._cond.notify_all()
            return cur

    def delete(self, key: str):
        with self._lock:
            self._store.pop(key, None)

    def clear(self):
        with self._lock:
            self._store.clear()

    def num_keys(self) -> int:
        return len(self._store)


class SyncService:
    """Named "all workers joined" syncs and notify-style barriers."""

    def __init__(self, job_manager=None):
        self._lock = threading.Lock()
        self._job_manager = job_manager
        self._syncs: Dict[str, Set[int]] = {}
        self._finished: Set[str] = set()
        self._barriers: Set[str] = set()

    def _expected(self) -> Set[int]:
        if self._job_manager is None:
            return set()
        return set(self._job_manager.running_node_ids())

    def join_sync(self, name: str, node_id: int) -> bool:
        with self._lock:
            self._syncs.setdefault(name, set()).add(node_id)
        return True

    def sync_finished(self, name: str) -> bool:
        with self._lock:
            if name in self._finished:
                return True
            joined = self._syncs.get(name, set())
            exp = self._expected()
            if exp and exp.issubset(joined):
                self._finished.add(name)
                return True
            return False

    def remove_exited_worker_sync(self, node_id: int):
        with self._lock:
            for s in self._syncs.values():
                s.discard(node_id)

    def notify_barrier(self, name: str) -> bool:
        with self._lock:
            self._barriers.add(name)
        return True

    def barrier(self, name: str) -> bool:
        with self._lock:
            return name in self._barriers


class SpeedMonitor:
    """Global-step records -> steps/s, and a worker-count stability check."""

    def __init__(self, window: int = 20):
        self._lock = threading.Lock()
        self._records: deque = deque(maxlen=window)  # (timestamp, step)
        self._workers: Set[int] = set()
        self._target_workers = 0
        self._init_time = time.time()
        self._first_step_time = 0.0
        self.completed_global_step = 0

    def set_target_worker_num(self, n: int):
        self._target_workers = n

    def add_running_worker(self, node_id: int):
        self._workers.add(node_id)

    def remove_running_worker(self, node_id: int):
        self._workers.discard(node_id)

    def collect_global_step(self, step: int, timestamp: float):
        with self._lock:
            if not self._first_step_time:
                self._first_step_time = timestamp
            if self._records and step <= self._records[-1][1]:
                # restarted from a checkpoint: reset the window
                self._records.clear()
            self._records.append((timestamp, step))
            self.completed_global_step = step

    def running_speed(self) -> float:
        with self._lock:
            if len(self._records) < 2:
                return 0.0
            (t0, s0), (t1, s1) = self._records[0], self._records[-1]
            return (s1 - s0) / (t1 - t0) if t1 > t0 else 0.0

    def worker_adjustment_finished(self) -> bool:
        return self._target_workers == 0 or len(self._workers) >= self._target_workers

    def last_step_time(self) -> float:
        with self._lock:
            return self._records[-1][0] if self._records else 0.0

    def reset(self):
        with self._lock:
            self._records.clear()


class ErrorMonitor:
    """Routes reported failures by level (reference error_monitor.py)."""

    def __init__(self, on_node_error=None):
        self._on_node_error = on_node_error
        self.records: List[Tuple[int, str, str]] = []

    def process_error(self, node_id: int, restart_count: int, error_data: str, level: str) -> bool:
        """Returns True if the node should be relaunched."""
        self.records.append((node_id, level, error_data[:2000]))
        if level == TrainingExceptionLevel.PROCESS_ERROR:
            logger.warning(f"process error on node {node_id} (restart {restart_count}): {error_data[:500]}")
            return False
        if level == TrainingExceptionLevel.NODE_ERROR:
            logger.error(f"node error on node {node_id}: {error_data[:500]}")
            if self._on_node_error:
                self._on_node_error(node_id, error_data)
            return True
        if level == TrainingExceptionLevel.RDZV_ERROR:
            logger.error(f"rendezvous error on node {node_id}: {error_data[:500]}")
            return False
        logger.info(f"[{level}] node {node_id}: {error_data[:500]}")
        return False


class DiagnosisManager:
    """Keeps a window of diagnosis data and runs the "training hang" check:
    no global-step progress for ``hang_secs`` while workers are running."""

    def __init__(self, speed_monitor: SpeedMonitor, hang_secs: float = 1800, window_secs: float = 600):
        self._speed = speed_monitor
        self._hang_secs = hang_secs
        self._window = window_secs
        self._data: deque = deque()
        self._lock = threading.Lock()

    def collect(self, node_id: int, data_cls: str, content: str, ts: Optional[float] = None):
        ts = ts or time.time()
        with self._lock:
            self._data.append((ts, node_id, data_cls, content))
            while self._data and ts - self._data[0][0] > self._window:
                self._data.popleft()

    def data(self, data_cls: Optional[str] = None):
        with self._lock:
            return [d for d in self._data if data_cls is None or d[2] == data_cls]

    def check_training_hang(self, now: Optional[float] = None) -> bool:
        now = now or time.time()
        last = self._speed.last_step_time()
        return bool(last) and now - last > self._hang_secs


class SimpleStrategyGenerator:
    """Suggests a dataloader batch size from free GPU memory (reference
    hyperparams/simple_strategy_generator.py)."""

    def __init__(self, gpu_memory_mb: int = 288 * 1024):
        self.gpu_memory_mb = gpu_memory_mb

    def generate(self, used_mb: int, batch_size: int, version: int = 0):
        from ..common.comm import DataLoaderConfig, OptimizerConfig, ParallelConfig

        if used_mb <= 0 or batch_size <= 0:
            return ParallelConfig(dataloader=DataLoaderConfig(version=version, batch_size=batch_size),
                                  optimizer=OptimizerConfig(version=version))
        per_sample = used_mb / batch_size
        free = self.gpu_memory_mb * 0.9 - used_mb
        extra = int(free // per_sample) if per_sample > 0 else 0
        new_bs = batch_size + max(0, extra)
        return ParallelConfig(dataloader=DataLoaderConfig(version=version + 1, batch_size=new_bs,
                                                          last_batch_size=batch_size),
                              optimizer=OptimizerConfig(version=version + 1))


class ElasticPsService:
    """Cluster versions for elastic parameter-server training.

    The *global* version counts PS-set changes (bumped by the master when a
    PS fails or is removed); each PS and worker reports the *local* version it
    is running with, and a worker the *restored* version its model state came
    from, so workers know when to rebuild their PS sessions.

    Parity: reference ``master/elastic_training/elastic_ps.py``
    (``ElasticPsService``) and ``servicer.py:173-187,478-490``.
    """

    def __init__(self):
        self._lock = threading.Lock()
        self.global_version = 0
        self._ps_local: Dict[int, int] = {}
        self._worker_local: Dict[int, int] = {}
        self._worker_restored: Dict[int, int] = {}

    def inc_global_cluster_version(self) -> int:
        with self._lock:
            self.global_version += 1
            logger.info(f"PS cluster global version -> {self.global_version}")
            return self.global_version

    def get_version(self, task_type: str, version_type: str, task_id: int) -> int:
        V = PSClusterVersionType
        with self._lock:
            if version_type == V.GLOBAL:
                return self.global_version
            if task_type == NodeType.PS and version_type == V.LOCAL:
                return self._ps_local.get(task_id, 0)
            if task_type == NodeType.WORKER and version_type == V.LOCAL:
                return self._worker_local.get(task_id, 0)
            if task_type == NodeType.WORKER and version_type == V.RESTORED:
                return self._worker_restored.get(task_id, -1)
        logger.warning(f"unsupported cluster version query {task_type}/{version_type}")
        return 0

    def update_version(self, task_type: str, version_type: str, task_id: int, version: int) -> bool:
        V = PSClusterVersionType
        with self._lock:
            if version_type == V.GLOBAL:
                self.global_version = version
            elif task_type == NodeType.PS and version_type == V.LOCAL:
                self._ps_local[task_id] = version
            elif task_type == NodeType.WORKER and version_type == V.LOCAL:
                self._worker_local[task_id] = version
            elif task_type == NodeType.WORKER and version_type == V.RESTORED:
                self._worker_restored[task_id] = version
            else:
                logger.warning(f"unsupported cluster version update {task_type}/{version_type}")
                return False
        return True

