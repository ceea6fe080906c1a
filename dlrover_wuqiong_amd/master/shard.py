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
import math
import os
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
    (``dataset_size`` <= 0) or until ``dataset_size`` records were issued.

    A stream may have several partitions (Kafka-style topics / files), each
    with its own next unconsumed offset; shards are cut round-robin over the
    partitions and ``ShardDef.name`` carries the partition name.  The offsets
    are part of the checkpoint (:meth:`to_checkpoint`), so a restored master
    resumes each partition where it stopped instead of replaying the stream
    from offset 0 (reference ``PartitionOffsets`` +
    ``StreamingDatasetSplitter.to_checkpoint/from_checkpoint``,
    ``dataset_splitter.py:43-88,414-440``)."""

    def __init__(self, *a, partition_offsets: Optional[Dict[str, int]] = None, shards_per_fetch: int = 16, **kw):
        super().__init__(*a, **kw)
        self.partition_offsets: Dict[str, int] = dict(partition_offsets or {self.dataset_name: 0})
        self._rr = 0  # next partition, round-robin
        self.issued = 0  # records handed out so far (bounded streams stop at dataset_size)
        self.shards_per_fetch = max(1, shards_per_fetch)

    @property
    def _offset(self) -> int:  # single-partition view (kept for callers/tests)
        return sum(self.partition_offsets.values())

    def epoch_finished(self):
        return self.dataset_size > 0 and self.issued >= self.dataset_size

    def create_shards(self):
        out = []
        parts = list(self.partition_offsets)
        for _ in range(self.shards_per_fetch):
            if self.epoch_finished():
                break
            name = parts[self._rr % len(parts)]
            self._rr += 1
            start = self.partition_offsets[name]
            n = self.shard_size
            if self.dataset_size > 0:
                n = min(n, self.dataset_size - self.issued)
            out.append(ShardDef(name, start, start + n))
            self.partition_offsets[name] = start + n
            self.issued += n
        return out

    def to_checkpoint(self) -> dict:
        return {"partition_offsets": dict(self.partition_offsets), "rr": self._rr, "issued": self.issued}

    def from_checkpoint(self, d: dict):
        if d.get("partition_offsets"):
            self.partition_offsets = {str(k): int(v) for k, v in d["partition_offsets"].items()}
        self._rr = int(d.get("rr", 0))
        self.issued = int(d.get("issued", 0))


MAX_TASK_RETRIES = int(os.environ.get("DWAMD_MAX_TASK_RETRIES", "3"))


class DatasetManager:
    def __init__(self, task_type: int, batch_size: int, splitter: DatasetSplitter,
                 max_task_retries: int = MAX_TASK_RETRIES):
        self.task_type = task_type
        self.batch_size = batch_size
        self.splitter = splitter
        self.todo: deque = deque()
        self.doing: Dict[int, tuple] = {}  # task_id -> (node_id, TaskDef, start_time)
        self._next_id = 0
        self.completed_steps = 0
        self.max_task_retries = max_task_retries
        self.failed_shards: List[ShardDef] = []  # dropped after max_task_retries failures

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

    def _requeue(self, t: TaskDef, why: str) -> bool:
        """Back to the todo queue unless the shard already failed
        ``max_task_retries`` times: then it is dropped with an error (a poison
        shard must not keep the job from ever finishing; reference
        ``_check_exceed_max_task_retries``, batch_dataset_manager.py:140-152)."""
        t.retry += 1
        if t.retry > self.max_task_retries:
            self.failed_shards.append(t.shard)
            logger.error(f"shard {t.shard.name}[{t.shard.start}:{t.shard.end}) dropped after "
                         f"{self.max_task_retries} retries (last: {why})")
            return False
        self.todo.appendleft(t)
        return True

    def report_task_status(self, task_id: int, success: bool) -> Optional[TaskDef]:
        item = self.doing.pop(task_id, None)
        if item is None:
            return None
        _node, t, _ts = item
        if success:
            n = t.shard.end - t.shard.start
            self.completed_steps += max(1, math.ceil(n / max(1, self.batch_size)))
        else:
            self._requeue(t, "reported failed")
        return t

    def recover_tasks(self, node_id: int):
        back = [tid for tid, (n, _t, _s) in self.doing.items() if n == node_id]
        for tid in back:
            _n, t, _s = self.doing.pop(tid)
            self._requeue(t, f"worker {node_id} died")
        return len(back)

    def reassign_timeout_tasks(self, timeout: float):
        now = time.time()
        late = [tid for tid, (_n, _t, s) in self.doing.items() if now - s > timeout]
        for tid in late:
            _n, t, _s = self.doing.pop(tid)
            self._requeue(t, f"not done within {timeout:.0f}s")
        return len(late)

    def finished(self) -> bool:
        return self.splitter.epoch_finished() and not self.todo and not self.doing

    def checkpoint(self) -> str:
        """Unfinished shards (todo + doing, with their retry counts), the
        epoch and the splitter's position (stream offsets)."""
        tasks = [t for t in self.todo] + [t for (_n, t, _s) in self.doing.values()]
        shards = [[t.shard.start, t.shard.end, t.shard.record_indices, t.shard.name, t.retry] for t in tasks]
        d = {"epoch": self.splitter.epoch, "todo": shards, "dataset_name": self.splitter.dataset_name,
             "completed_steps": self.completed_steps}
        if hasattr(self.splitter, "to_checkpoint"):
            d["splitter"] = self.splitter.to_checkpoint()
        return json.dumps(d)

    def restore_checkpoint(self, content: str):
        d = json.loads(content)
        self.splitter.epoch = d.get("epoch", 0)
        if "splitter" in d and hasattr(self.splitter, "from_checkpoint"):
            self.splitter.from_checkpoint(d["splitter"])
        self.completed_steps = int(d.get("completed_steps", self.completed_steps))
        self.todo.clear()
        self.doing.clear()
        for item in d.get("todo", []):
            s, e, idx = item[:3]
            name = item[3] if len(item) > 3 else d["dataset_name"]
            t = TaskDef(self._alloc_id(), self.task_type, ShardDef(name, s, e, idx))
            t.retry = int(item[4]) if len(item) > 4 else 0
            self.todo.append(t)


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
                    storage_type: str = "table", partition_offsets: Optional[Dict[str, int]] = None):
        with self._lock:
            if dataset_name in self._datasets:
                return
            shard_size = batch_size * max(1, num_minibatches_per_shard)
            if storage_type == "stream":
                splitter = StreamingDatasetSplitter(dataset_name, dataset_size, shard_size, num_epochs, shuffle,
                                                    partition_offsets=partition_offsets)
            else:
                cls = TextDatasetSplitter if storage_type == "text" else TableDatasetSplitter
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
