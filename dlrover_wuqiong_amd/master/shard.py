"""Dynamic data sharding (master side).

The dataset is cut into small shards (``batch_size * num_minibatches_per_shard``
records); workers pull a shard when they finish the previous one, so a slow
worker simply pulls fewer shards and a failed worker's in-flight shards go
back to the todo queue.  Shard progress is checkpointable.

Parity: reference ``dlrover/python/master/shard/`` (``task_manager.py:37-297``,
``dataset_splitter.py:90-481`` table/text/streaming splitters,
``batch_dataset_manager.py:29``, ``streaming_dataset_manager.py:32``).
"""

import json
import random
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..common.log import logger


class TaskType:
    NONE = 0
    TRAINING = 1
    EVALUATION = 2
    PREDICTION = 3
    WAIT = 4


@dataclass
class ShardDef:
    name: str
    start: int
    end: int
    record_indices: List[int] = field(default_factory=list)


@dataclass
class TaskDef:
    task_id: int
    task_type: int
    shard: ShardDef
    retry: int = 0


class DatasetSplitter:
    def __init__(self, dataset_name: str, dataset_size: int, shard_size: int, num_epochs: int = 1,
                 shuffle: bool = False):
        self.dataset_name = dataset_name
        self.dataset_size = dataset_size
        self.shard_size = max(1, shard_size)
        self.num_epochs = num_epochs
        self.shuffle = shuffle
        self.epoch = 0

    def epoch_finished(self) -> bool:
        return self.epoch >= self.num_epochs

    def create_shards(self) -> List[ShardDef]:
        raise NotImplementedError


class TableDatasetSplitter(DatasetSplitter):
    """Contiguous [start, end) ranges of a table; shuffle permutes shards."""

    def create_shards(self):
        shards = [ShardDef(self.dataset_name, s, min(s + self.shard_size, self.dataset_size))
                  for s in range(0, self.dataset_size, self.shard_size)]
        if self.shuffle:
            random.shuffle(shards)
        self.epoch += 1
        return shards


class TextDatasetSplitter(DatasetSplitter):
    """Shards carry explicit record indices (shuffled within the epoch)."""

    def create_shards(self):
        idx = list(range(self.dataset_size))
        if self.shuffle:
            random.shuffle(idx)
        shards = []
        for s in range(0, self.dataset_size, self.shard_size):
            part = idx[s:s + self.shard_size]
            shards.append(ShardDef(self.dataset_name, s, s + len(part), part))
        self.epoch += 1
        return shards


class StreamingDatasetSplitter(DatasetSplitter):
    """Unbounded stream: hands out the next ``shard_size`` offsets forever
    (``dataset_size`` <= 0) or until ``dataset_size``."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self._offset = 0

    def epoch_finished(self):
        return self.dataset_size > 0 and self._offset >= self.dataset_size

    def create_shards(self):
        n = 16
        out = []
        for _ in range(n):
            if self.dataset_size > 0 and self._offset >= self.dataset_size:
                break
            end = self._offset + self.shard_size
            if self.dataset_size > 0:
                end = min(end, self.dataset_size)
            out.append(ShardDef(self.dataset_name, self._offset, end))
            self._offset = end
        return out


class DatasetManager:
    def __init__(self, task_type: int, batch_size: int, splitter: DatasetSplitter):
        self.task_type = task_type
        self.batch_size = batch_size
        self.splitter = splitter
        self.todo: deque = deque()
        self.doing: Dict[int, tuple] = {}  # task_id -> (node_id, TaskDef, start_time)
        self._next_id = 0
        self.completed_steps = 0

    def get_task(self, node_id: int) -> Optional[TaskDef]:
        if not self.todo and not self.splitter.epoch_finished():
            for s in self.splitter.create_shards():
                self.todo.append(TaskDef(self._alloc_id(), self.task_type, s))
        if not self.todo:
            return None
        t = self.todo.popleft()
        self.doing[t.task_id] = (node_id, t, time.time())
        return t

    def _alloc_id(self):
        self._next_id += 1
        return self._next_id

    def report_task_status(self, task_id: int, success: bool) -> Optional[TaskDef]:
        item = self.doing.pop(task_id, None)
        if item is None:
            return None
        _node, t, _ts = item
        if success:
            n = t.shard.end - t.shard.start
            self.completed_steps += max(1, n // max(1, self.batch_size))
        else:
            t.retry += 1
            self.todo.appendleft(t)
        return t

    def recover_tasks(self, node_id: int):
        back = [tid for tid, (n, _t, _s) in self.doing.items() if n == node_id]
        for tid in back:
            _n, t, _s = self.doing.pop(tid)
            self.todo.appendleft(t)
        return len(back)

    def reassign_timeout_tasks(self, timeout: float):
        now = time.time()
        late = [tid for tid, (_n, _t, s) in self.doing.items() if now - s > timeout]
        for tid in late:
            _n, t, _s = self.doing.pop(tid)
            self.todo.appendleft(t)
        return len(late)

    def finished(self) -> bool:
        return self.splitter.epoch_finished() and not self.todo and not self.doing

    def checkpoint(self) -> str:
        shards = [[t.shard.start, t.shard.end, t.shard.record_indices] for t in self.todo]
        shards += [[t.shard.start, t.shard.end, t.shard.record_indices] for (_n, t, _s) in self.doing.values()]
        return json.dumps({"epoch": self.splitter.epoch, "todo": shards,
                           "dataset_name": self.splitter.dataset_name})

    def restore_checkpoint(self, content: str):
        d = json.loads(content)
        self.splitter.epoch = d.get("epoch", 0)
        self.todo.clear()
        self.doing.clear()
        for s, e, idx in d.get("todo", []):
            self.todo.append(TaskDef(self._alloc_id(), self.task_type, ShardDef(d["dataset_name"], s, e, idx)))


class TaskManager:
    """Owns every dataset's shard queue; recovers shards of dead workers and
    reassigns shards that were held longer than ``task_timeout``."""

    def __init__(self, task_timeout: float = 1800.0):
        self._lock = threading.Lock()
        self._datasets: Dict[str, DatasetManager] = {}
        self.task_timeout = task_timeout
        self._worker_start_task_time: Dict[int, float] = {}

    def new_dataset(self, batch_size: int, dataset_size: int, dataset_name: str, num_epochs: int = 1,
                    shuffle: bool = False, num_minibatches_per_shard: int = 1, task_type: int = TaskType.TRAINING,
                    storage_type: str = "table"):
        with self._lock:
            if dataset_name in self._datasets:
                return
            shard_size = batch_size * max(1, num_minibatches_per_shard)
            cls = {"text": TextDatasetSplitter, "stream": StreamingDatasetSplitter}.get(storage_type,
                                                                                        TableDatasetSplitter)
            splitter = cls(dataset_name, dataset_size, shard_size, num_epochs, shuffle)
            self._datasets[dataset_name] = DatasetManager(task_type, batch_size, splitter)
            logger.info(f"dataset {dataset_name}: size={dataset_size} shard={shard_size} epochs={num_epochs}")

    def get_dataset(self, name) -> Optional[DatasetManager]:
        return self._datasets.get(name)

    def get_dataset_task(self, node_id: int, dataset_name: str) -> Optional[TaskDef]:
        with self._lock:
            ds = self._datasets.get(dataset_name)
            if ds is None:
                return None
            self._worker_start_task_time[node_id] = time.time()
            return ds.get_task(node_id)

    def report_dataset_task(self, dataset_name: str, task_id: int, success: bool):
        with self._lock:
            ds = self._datasets.get(dataset_name)
            return ds.report_task_status(task_id, success) if ds else None

    def recover_tasks(self, node_id: int) -> int:
        with self._lock:
            return sum(ds.recover_tasks(node_id) for ds in self._datasets.values())

    def reassign_timeout_tasks(self) -> int:
        with self._lock:
            return sum(ds.reassign_timeout_tasks(self.task_timeout) for ds in self._datasets.values())

    def finished(self) -> bool:
        return bool(self._datasets) and all(ds.finished() for ds in self._datasets.values())

    def get_dataset_checkpoint(self, name: str) -> str:
        ds = self._datasets.get(name)
        return ds.checkpoint() if ds else ""

    def restore_dataset_from_checkpoint(self, content: str) -> bool:
        try:
            d = json.loads(content)
        except Exception:
            return False
        ds = self._datasets.get(d.get("dataset_name", ""))
        if ds is None:
            return False
        ds.restore_checkpoint(content)
        return True

    def training_started(self) -> bool:
        return bool(self._worker_start_task_time)
